// mm2rs — command line of the MI355X path, flag-compatible with the
// reference CLI (src/main.rs:11-233):
//   mm2rs index <ref.fa> [-w 10] [-k 15] [-b 14] [-H] [-d out.mmi]
//   mm2rs align <ref.mmi|ref.fa> <reads.fa> [-w] [-k] [-H] [-f] [-g] [-r bw[,bw_long]]
//               [-n] [-m] [-M] [-p] [-N] [-x preset] [-a] [-o out]
// Extra flags: -t threads (host index build), --device N, --batch-bases N,
// --first-only (map only the first record, exactly as the reference does).
// Unlike the reference, align maps every record of <reads.fa>; the output is
// the per-read concatenation of what the reference prints for each read alone.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mm2g.h"
#include "mm2g_index.h"

static void usage() {
    fprintf(stderr,
            "Usage: mm2rs index <fasta> [-w 10] [-k 15] [-b 14] [-H] [-d out.mmi] [-t threads] [--device N] [--cpu-index]\n"
            "       mm2rs align <ref.mmi|ref.fa> <reads.fa> [-w 10] [-k 15] [-H] [-f 2e-4] [-g 5000] [-r bw[,bw_long]]\n"
            "                   [-n 3] [-m 40] [-M 0.5] [-p 0.8] [-N 5] [-x map-ont|map-hifi|lr:hq|sr] [-a] [-o out]\n"
            "                   [-t threads] [--device N] [--batch-bases N] [--first-only]\n");
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
        else if (a == "--batch-bases") batch_bases = atoll(nxt().c_str());
        else if (a == "--first-only") first_only = true;
        else if (a == "--cpu-index") cpu_index = true;
        else if (!a.empty() && a[0] == '-' && a.size() > 1) { fprintf(stderr, "error: unknown option %s\n", a.c_str()); usage(); return 2; }
        else pos.push_back(a);
    }
    if (cmd == "index") {   // main.rs:150-159
        if (pos.size() != 1) { usage(); return 2; }
        const int flag = hpc ? 1 : 0;
        mm2g_index* idx = nullptr;
        const bool gpu = !cpu_index && mm2g_device_count() > 0;
        const int st0 = gpu ? mm2g_index_build_fasta_gpu(pos[0].c_str(), w, k, b, flag, device, threads, &idx)
                            : mm2g_index_build_fasta(pos[0].c_str(), w, k, b, flag, threads, &idx);
        if (st0 != 0) { fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1; }
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
    if (cmd != "align") { usage(); return 2; }
    if (pos.size() != 2) { usage(); return 2; }
    // apply_preset (main.rs:125-133)
    if (preset == "map-ont") { k = 15; w = 10; }
    else if (preset == "map-hifi" || preset == "lr:hq") { k = 19; w = 10; }
    else if (preset == "sr") { k = 21; w = 11; }
    mo.w = w; mo.k = k;
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
    int32_t mid_occ;
    mm2g_index_calc_mid_occ(idx, frac, &mid_occ);
    if (mid_occ < 10) mid_occ = 10;                        // main.rs:197
    mm2g_ctx* ctx = nullptr;
    if (mm2g_ctx_create(device, &ctx) != 0 || mm2g_ctx_upload_index(ctx, idx, mid_occ) != 0) {
        fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1;
    }
    std::vector<mm2g::FastaRecord> recs; std::string err;
    if (!mm2g::read_fasta(pos[1].c_str(), recs, first_only, err)) { fprintf(stderr, "Error: %s\n", err.c_str()); return 1; }
    FILE* fo = stdout;
    if (!out.empty() && out != "-") { fo = fopen(out.c_str(), "w"); if (!fo) { fprintf(stderr, "Error: cannot create %s\n", out.c_str()); return 1; } }
    std::vector<char> pafbuf;
    for (size_t r0 = 0; r0 < recs.size();) {
        size_t r1 = r0; long long bases = 0;
        while (r1 < recs.size() && (r1 == r0 || bases + (long long)recs[r1].seq.size() <= batch_bases)) { bases += (long long)recs[r1].seq.size(); ++r1; }
        std::vector<uint64_t> offs(r1 - r0 + 1, 0);
        std::string cat; cat.reserve((size_t)bases);
        std::vector<const char*> names;
        for (size_t i = r0; i < r1; ++i) { cat += recs[i].seq; offs[i - r0 + 1] = cat.size(); names.push_back(recs[i].name.c_str()); }
        const uint32_t n = (uint32_t)(r1 - r0);
        std::vector<mm2g_read_result> res(n);
        if (mm2g_batch_set_reads(ctx, (const uint8_t*)cat.data(), offs.data(), n) != 0 || mm2g_batch_map(ctx, &mo) != 0 ||
            mm2g_batch_results(ctx, res.data(), n) != 0) {
            fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1;
        }
        for (uint32_t i = 0; i < n; ++i) {
            if (res[i].flags & MM2G_R_EMPTY) fprintf(stderr, "warning: read %s is empty (the reference asserts on it, src/sketch.rs:40); skipped\n", names[i]);
            if (res[i].flags & MM2G_R_PANIC) fprintf(stderr, "warning: read %s: the reference panics here (index out of bounds: rid 2147483647, DESIGN.md Q19); no PAF line\n", names[i]);
        }
        int64_t need = mm2g_format_paf(idx, res.data(), names.data(), n, nullptr, 0);
        pafbuf.resize((size_t)need + 512 * n + 1);
        int64_t got = mm2g_format_paf(idx, res.data(), names.data(), n, pafbuf.data(), (int64_t)pafbuf.size());
        if (got < 0) { fprintf(stderr, "Error: %s\n", mm2g_last_error()); return 1; }
        fwrite(pafbuf.data(), 1, (size_t)got, fo);
        r0 = r1;
    }
    if (fo != stdout) fclose(fo);
    mm2g_ctx_destroy(ctx);
    mm2g_index_free(idx);
    return 0;
}
