// mm2rs — command line of the MI355X path, flag-compatible with the
// reference CLI (src/main.rs:11-233):
//   mm2rs index <ref.fa> [-w 10] [-k 15] [-b 14] [-H] [-d out.mmi]
//   mm2rs align <ref.mmi|ref.fa> <reads.fa|fq> [-w] [-k] [-H] [-f] [-g] [-r bw[,bw_long]]
//               [-n] [-m] [-M] [-p] [-N] [-x preset] [-a] [-o out]
//   mm2rs anchors <ref> <reads.fa> [-w] [-k] [-H]       (main.rs:160-171)
//   mm2rs chain <ref> <reads.fa> [-w] [-k] [-r 5000] [-H] (main.rs:172-186)
// Extra flags: -t threads (host index build), --device N, --devices 0,1,..,
// --batch-bases N, --streams N (contexts per GPU in the align pipeline),
// --first-only (map only the first record, exactly as the reference does),
// --cpu-index.
// Unlike the reference, align maps every record of <reads> (FASTA or FASTQ),
// streaming: a reader fills batches, N contexts per GPU (HIP streams, one
// device index per GPU, the GPUs' copies uploaded in parallel) pull them from
// one queue -- batch k+1's upload and sketch overlap batch k's chaining, and
// reads shard over the GPUs of --devices -- and a writer emits PAF in input
// order.  The output is the per-read concatenation of what the reference
// prints for each read alone (src/main.rs:189-230), whatever the device count.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <condition_variable>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mm2g.h"
#include "mm2g_index.h"

static void usage() {
    fprintf(stderr,
            "Usage: mm2rs index <fasta> [-w 10] [-k 15] [-b 14] [-H] [-d out.mmi] [-t threads] [--device N] [--cpu-index]\n"
            "       mm2rs align <ref.mmi|ref.fa> <reads.fa> [-w 10] [-k 15] [-H] [-f 2e-4] [-g 5000] [-r bw[,bw_long]]\n"
            "                   [-n 3] [-m 40] [-M 0.5] [-p 0.8] [-N 5] [-x map-ont|map-hifi|lr:hq|sr] [-a] [-o out]\n"
            "                   [-t threads] [--device N | --devices 0,1,..] [--streams N] [--batch-bases N] [--first-only]\n");
}

static bool ends_with(const std::string& s, const char* suf) {
    size_t n = strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

int main(int argc, char** argv) {
    if (argc < 2) { usage(); return 2; }
    std::string cmd = argv[1];
    std::vector<std::string> pos;
    int w = 10, k = 15, b = 14, threads = 8, device = 0;
    bool hpc = false, first_only = false, cpu_index = false;
    float frac = 2e-4f;
    std::string dump, out, preset, ropt;
    mm2g_map_opts mo; mm2g_map_opts_default(&mo);
    long long batch_bases = 256LL << 20;
    int n_streams = 4;
    std::vector<int> devices;
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        auto nxt = [&]() -> std::string { if (i + 1 >= argc) { usage(); exit(2); } return std::string(argv[++i]); };
        if (a == "-w") w = atoi(nxt().c_str());
        else if (a == "-k") k = atoi(nxt().c_str());
        else if (a == "-b") b = atoi(nxt().c_str());
        else if (a == "-H" || a == "--hpc") hpc = true;
        else if (a == "-d" || a == "--dump") dump = nxt();
        else if (a == "-f") frac = (float)atof(nxt().c_str());
        else if (a == "-g") mo.max_gap = atoi(nxt().c_str());
        else if (a == "-r") ropt = nxt();
        else if (a == "-n") mo.min_cnt = atoi(nxt().c_str());
        else if (a == "-m") mo.min_chain_score = atoi(nxt().c_str());
        else if (a == "-M" || a == "--mask-level") mo.mask_level = (float)atof(nxt().c_str());
        else if (a == "-p" || a == "--pri-ratio") mo.pri_ratio = (float)atof(nxt().c_str());
        else if (a == "-N" || a == "--best-n") mo.best_n = atoi(nxt().c_str());
        else if (a == "-x") preset = nxt();
        else if (a == "-a") {}
        else if (a == "-o") out = nxt();
        else if (a == "-t") threads = atoi(nxt().c_str());
        else if (a == "--device") device = atoi(nxt().c_str());
        else if (a == "--devices") {   // comma-separated device ids; a device may repeat (one index copy each)
            devices.clear();
            const std::string v = nxt();
            for (size_t p = 0; p <= v.size();) {
                size_t q = v.find(',', p);
                if (q == std::string::npos) q = v.size();
                const std::string t = v.substr(p, q - p);
                char* e; const long d = strtol(t.c_str(), &e, 10);
                if (t.empty() || *e || d < 0) { fprintf(stderr, "error: --devices expects a list like 0,1,2\n"); return 2; }
                devices.push_back((int)d);
                p = q + 1;
            }
        }
        else if (a == "--batch-bases") batch_bases = atoll(nxt().c_str());
        else if (a == "--streams") n_streams = std::max(1, atoi(nxt().c_str()));
        else if (a == "--first-only") first_only = true;
        else if (a == "--cpu-index") cpu_index = true;
        else if (!a.empty() && a[0] == '-' && a.size() > 1) { fprintf(stderr, "error: unknown option %s\n", a.c_str()); usage(); return 2; }
        else pos.push_back(a);
    }
    if (!devices.empty()) device = devices[0];
    if (cmd == "index") {   // main.rs:150-159
        if (pos.size() != 1) { usage(); return 2; }
        const int flag = hpc ? 1 : 0;
        mm2g_index* idx = nullptr;
        const bool gpu = !cpu_index && mm2g_device_count() > 0;
        const int st0 = gpu ? mm2g_index_build_fasta_gpu(pos[0].c_str(), w, k, b, flag, device, threads, &idx)
                            : mm2g_index_build_fasta(pos[0].c_str(), w, k, b, flag, threads, &idx);
        if (st0 != 0) { fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1; }
        const char* why = nullptr;
        if (mm2g_index_origin(idx, &why) == MM2G_IX_GPU_FALLBACK)
            fprintf(stderr, "warning: the GPU index build fell back to the host build (%s); the index is the same\n", why ? why : "?");
        uint64_t nk, tl; double ao, as; uint32_t n_seq;
        mm2g_index_stats(idx, &nk, &ao, &as, &tl);
        mm2g_index_params(idx, nullptr, nullptr, nullptr, nullptr, &n_seq);
        printf("kmer size: %d; skip: %d; is_hpc: %d; #seq: %u\n", k, w, hpc ? 1 : 0, n_seq);
        printf("distinct minimizers: %llu (avg occ %.2f) avg spacing %.3f total length %llu\n", (unsigned long long)nk, ao, as, (unsigned long long)tl);
        if (!dump.empty()) {
            if (!ends_with(dump, ".mmi")) { fprintf(stderr, "Error: only minimap2 .mmi dumps are supported (the MM2RSIDX format is out of scope)\n"); mm2g_index_free(idx); return 1; }
            if (mm2g_index_save_mmi(idx, dump.c_str()) != 0) { fprintf(stderr, "Error: %s\n", mm2g_last_error()); mm2g_index_free(idx); return 1; }
        }
        mm2g_index_free(idx);
        return 0;
    }
    if (cmd != "align" && cmd != "anchors" && cmd != "chain") { usage(); return 2; }
    const bool dbg_cmd = cmd != "align";
    if (dbg_cmd) { preset.clear(); }
    if (pos.size() != 2) { usage(); return 2; }
    // apply_preset (main.rs:125-133)
    if (preset == "map-ont") { k = 15; w = 10; }
    else if (preset == "map-hifi" || preset == "lr:hq") { k = 19; w = 10; }
    else if (preset == "sr") { k = 21; w = 11; }
    mo.w = w; mo.k = k;
    if (cmd == "chain") {   // Chain: default_chain_params(k) with bw = -r (default 5000), chain_dp (no rescue)
        mo.bw = ropt.empty() ? 5000 : atoi(ropt.c_str());
        ropt.clear();
    }
    if (!ropt.empty()) {   // main.rs:202-207: "-r bw[,bw_long]", unparsable parts ignored
        size_t c = ropt.find(',');
        std::string a0 = ropt.substr(0, c);
        char* e; long v = strtol(a0.c_str(), &e, 10);
        if (!a0.empty() && *e == 0) mo.bw = (int)v;
        if (c != std::string::npos) { std::string a1 = ropt.substr(c + 1); v = strtol(a1.c_str(), &e, 10); if (!a1.empty() && *e == 0) mo.bw_long = (int)v; }
    }
    // load_index_auto (main.rs:135-145) with b = 14 (main.rs:192)
    mm2g_index* idx = nullptr;
    const std::string& ref = pos[0];
    int st;
    if (ends_with(ref, ".mmi")) st = mm2g_index_load_mmi(ref.c_str(), &idx);
    else {
        FILE* f = fopen(ref.c_str(), "rb"); char m[9] = {0};
        if (f) { size_t got = fread(m, 1, 9, f); fclose(f); if (got == 9 && memcmp(m, "MM2RSIDX\0", 9) == 0) { fprintf(stderr, "Error: MM2RSIDX indexes are out of scope; use .mmi\n"); return 1; } }
        st = (!cpu_index && mm2g_device_count() > 0) ? mm2g_index_build_fasta_gpu(ref.c_str(), w, k, 14, hpc ? 1 : 0, device, threads, &idx)
                                                     : mm2g_index_build_fasta(ref.c_str(), w, k, 14, hpc ? 1 : 0, threads, &idx);
    }
    if (st != 0) { fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1; }
    {
        const char* why = nullptr;
        if (mm2g_index_origin(idx, &why) == MM2G_IX_GPU_FALLBACK)
            fprintf(stderr, "warning: the GPU index build fell back to the host build (%s); the index is the same\n", why ? why : "?");
    }
    if (devices.empty() || dbg_cmd) devices.assign(1, device);
    {
        const int nd = mm2g_device_count();
        for (int d : devices)
            if (d >= nd) { fprintf(stderr, "Error: device %d out of range (%d devices visible)\n", d, nd); return 1; }
    }
    // one index copy per listed device, uploaded in parallel; calc_mid_occ
    // (main.rs:196-197) on the first device's table
    int32_t mid_occ = 10;
    std::vector<mm2g_ctx*> heads(devices.size(), nullptr);
    for (size_t i = 0; i < devices.size(); ++i)
        if (mm2g_ctx_create(devices[i], &heads[i]) != 0) { fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1; }
    if (mm2g_ctx_upload_index_many(heads.data(), (int)heads.size(), idx, mid_occ) != 0 ||
        mm2g_ctx_index_mid_occ(heads[0], frac, &mid_occ) != 0) {
        fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1;
    }
    if (mid_occ < 10) mid_occ = 10;                        // main.rs:197
    for (mm2g_ctx* h : heads) mm2g_ctx_set_mid_occ(h, mid_occ);
    mm2g_ctx* ctx = heads[0];
    if (dbg_cmd) {   // anchors / chain of the first read (read_fasta_first, main.rs:92-103)
        mm2g::SeqStream in; std::string err;
        mm2g::FastaRecord rec;
        if (!in.open(pos[1].c_str(), err)) { fprintf(stderr, "Error: %s\n", err.c_str()); return 1; }
        if (!in.next(rec)) rec = mm2g::FastaRecord{"*", std::string()};
        mm2g_ctx_set_debug(ctx, 1);   // full sorted anchors and f / pprev
        if (cmd == "chain") mo.bw_long = mo.bw;   // a rescue pass with the same parameters = chain_dp
        uint64_t offs[2] = {0, rec.seq.size()};
        mm2g_read_result res;
        if (mm2g_batch_set_reads(ctx, (const uint8_t*)rec.seq.data(), offs, 1) != 0 || mm2g_batch_map(ctx, &mo) != 0 ||
            mm2g_batch_results(ctx, &res, 1) != 0) { fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1; }
        const int64_t A = mm2g_debug_anchors(ctx, 0, nullptr, 0);
        std::vector<uint64_t> xy((size_t)std::max<int64_t>(A, 1) * 2);
        if (A > 0) mm2g_debug_anchors(ctx, 0, xy.data(), A);
        if (cmd == "anchors") {
            printf("anchors: %lld\n", (long long)A);
            for (int64_t i = 0; i < A && i < 10; ++i) printf("x=0x%016llx y=0x%016llx\n", (unsigned long long)xy[2 * i], (unsigned long long)xy[2 * i + 1]);
        } else {
            // fallback chain (lchain.rs:162-171): last argmax f, pprev walk
            std::vector<int32_t> f((size_t)std::max<int64_t>(A, 1)), pp((size_t)std::max<int64_t>(A, 1));
            if (A > 0) mm2g_debug_dp(ctx, 0, f.data(), pp.data(), A);
            std::vector<int64_t> ch;
            if (A > 0) {
                int64_t bi = 0;
                for (int64_t i = 1; i < A; ++i) if (f[i] >= f[bi]) bi = i;
                for (int64_t i = bi; i >= 0; i = pp[i]) ch.push_back(i);
            }
            printf("best_chain_len: %zu\n", ch.size());
            if (!ch.empty()) {
                const int64_t st = ch.back(), en = ch.front();
                printf("start: x=0x%016llx y=0x%016llx\n", (unsigned long long)xy[2 * st], (unsigned long long)xy[2 * st + 1]);
                printf("end:   x=0x%016llx y=0x%016llx\n", (unsigned long long)xy[2 * en], (unsigned long long)xy[2 * en + 1]);
            }
        }
        for (mm2g_ctx* h : heads) mm2g_ctx_destroy(h);
        mm2g_index_free(idx);
        return 0;
    }
    // ---- streaming align: reader -> N mapping contexts per GPU -> in-order writer
    std::vector<mm2g_ctx*> ctxs;
    for (int i = 0; i < n_streams; ++i)      // interleaved over the GPUs, so each starts working at once
        for (size_t d = 0; d < heads.size(); ++d) {
            mm2g_ctx* c2 = heads[d];
            if (i > 0 && (mm2g_ctx_create(devices[d], &c2) != 0 || mm2g_ctx_share_index(c2, heads[d], mid_occ) != 0)) {
                fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1;
            }
            ctxs.push_back(c2);
        }
    mm2g::SeqStream in; std::string err;
    if (!in.open(pos[1].c_str(), err)) { fprintf(stderr, "Error: %s\n", err.c_str()); return 1; }
    FILE* fo = stdout;
    if (!out.empty() && out != "-") { fo = fopen(out.c_str(), "w"); if (!fo) { fprintf(stderr, "Error: cannot create %s\n", out.c_str()); return 1; } }
    struct Batch {
        size_t no = 0;
        std::vector<std::string> names;
        std::string cat;
        std::vector<uint64_t> offs{0};
        std::vector<mm2g_read_result> res;
        std::vector<char> paf;                // formatted by the worker (mm2g_batch_paf reads its context)
        bool ok = false;
    };
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Batch*> todo;                 // FIFO of batches to map
    std::map<size_t, Batch*> done;            // mapped, by batch number
    bool eof = false, failed = false;
    size_t n_batches = 0;
    const size_t max_inflight = 2 * ctxs.size() + 1;
    size_t inflight = 0;
    auto worker = [&](mm2g_ctx* c) {
        for (;;) {
            Batch* B;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !todo.empty() || eof || failed; });
                if (todo.empty()) return;
                B = todo.front(); todo.erase(todo.begin());
            }
            const uint32_t n = (uint32_t)B->names.size();
            B->res.resize(n);
            B->ok = mm2g_batch_set_reads(c, (const uint8_t*)B->cat.data(), B->offs.data(), n) == 0 && mm2g_batch_map(c, &mo) == 0 &&
                    mm2g_batch_results(c, B->res.data(), n) == 0;
            if (B->ok) {   // write_paf_many_with_scores (paf.rs:238-248): one line per read, or several under -n <= 1 -m <= k
                std::vector<const char*> nm(n);
                for (uint32_t i = 0; i < n; ++i) nm[i] = B->names[i].c_str();
                const int64_t need = mm2g_batch_paf(c, nm.data(), n, nullptr, 0);
                B->paf.resize((size_t)std::max<int64_t>(need, 0) + 1);
                const int64_t got = need < 0 ? need : mm2g_batch_paf(c, nm.data(), n, B->paf.data(), (int64_t)B->paf.size());
                B->ok = got >= 0;
                if (B->ok) B->paf.resize((size_t)got);
            }
            if (!B->ok) fprintf(stderr, "Error: %s\n", mm2g_last_error());
            {
                std::lock_guard<std::mutex> lk(mu);
                done[B->no] = B;
                if (!B->ok) failed = true;
            }
            cv.notify_all();
        }
    };
    auto writer = [&]() {
        for (size_t next = 0;; ++next) {
            Batch* B;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return done.count(next) || (eof && next >= n_batches) || failed; });
                if (!done.count(next)) return;
                B = done[next]; done.erase(next);
            }
            if (B->ok) {
                const uint32_t n = (uint32_t)B->names.size();
                for (uint32_t i = 0; i < n; ++i) {
                    const char* nm = B->names[i].c_str();
                    if (B->res[i].flags & MM2G_R_EMPTY) fprintf(stderr, "warning: read %s is empty (the reference asserts on it, src/sketch.rs:30); skipped\n", nm);
                    if (B->res[i].flags & MM2G_R_PANIC) fprintf(stderr, "warning: read %s: the reference panics here (index out of bounds: rid 2147483647 (DESIGN.md Q19), or an empty chain under -n <= 0); no PAF line\n", nm);
                }
                fwrite(B->paf.data(), 1, B->paf.size(), fo);
            }
            delete B;
            { std::lock_guard<std::mutex> lk(mu); --inflight; }
            cv.notify_all();
        }
    };
    std::vector<std::thread> th;
    for (mm2g_ctx* c : ctxs) th.emplace_back(worker, c);
    std::thread wt(writer);
    {   // reader: batches of up to --batch-bases bases (at least one read)
        mm2g::FastaRecord rec;
        Batch* B = nullptr;
        size_t n_read = 0;
        auto push = [&](Batch* b) {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return inflight < max_inflight || failed; });
            b->no = n_batches++; ++inflight;
            todo.push_back(b);
            cv.notify_all();
        };
        while (!(first_only && n_read >= 1) && in.next(rec)) {
            ++n_read;
            if (B && !B->names.empty() && (long long)(B->cat.size() + rec.seq.size()) > batch_bases) { push(B); B = nullptr; }
            if (!B) B = new Batch();
            B->names.push_back(rec.name);
            B->cat += rec.seq;
            B->offs.push_back(B->cat.size());
            { std::lock_guard<std::mutex> lk(mu); if (failed) break; }
        }
        if (B) push(B);
        { std::lock_guard<std::mutex> lk(mu); eof = true; }
        cv.notify_all();
    }
    for (auto& t : th) t.join();
    { std::lock_guard<std::mutex> lk(mu); eof = true; }
    cv.notify_all();
    wt.join();
    if (fo != stdout) fclose(fo);
    for (mm2g_ctx* c : ctxs) mm2g_ctx_destroy(c);
    mm2g_index_free(idx);
    return failed ? 1 : 0;
}
