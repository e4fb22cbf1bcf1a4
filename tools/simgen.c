// simgen — seeded synthetic references and ONT-shaped reads.
//
// There are no genomes in this container or on the GPU box, so every
// benchmark and parity input is synthetic.  RNG: xoshiro256** seeded through
// splitmix64; every contig gets its own stream (seed, contig index), so the
// output is identical for any thread count.
//
// Presets:
//   hg38   24 contigs with the GRCh38 primary lengths (sum 3.09 Gb), GC 41 %,
//          Alu-like 300 bp copies (~10 %, 10-15 % divergence), L1-like
//          fragments of a 6 kb consensus (~17 %, 5-20 %), a 171 bp satellite
//          array (~3 %), segmental duplications 10-100 kb (~5 %, 1-4 %),
//          10 kb N telomeres and a 50 kb N gap; repeats soft-masked
//          (lowercase), as hg38 is.
//   ecoli  1 contig of 4,641,652 bp, GC 50.8 %, 1 % IS-like 1.3 kb copies.
//   chr8chr12  hg38 chr8 + chr12 lengths (145 + 133 Mb), hg38-shaped (config C1).
//   small  3 contigs (60, 45, 30 kb) shaped like hg38 (fixtures / unit tests).
//   scale  multiplies every contig length (hg38 at scale 0.01 = 31 Mb).
//
// Reads (ONT-shaped): uniform start on an N-free template, 50 % reverse
// complemented, 8 % errors (3.5 % substitution, 2.25 % insertion of which
// half copy the neighbouring base, 2.25 % deletion), 0.05 % of reads carry a
// 20-N run, names r<idx>.
//
// Library C-ABI (ctypes from bench.py / tests) + CLI (`simgen genome|reads`).
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t s[4]; } rng_t;
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t splitmix64(uint64_t* x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static void rng_seed(rng_t* r, uint64_t seed, uint64_t stream) {
    uint64_t x = seed * 0x9E3779B97F4A7C15ULL ^ (stream + 0x632BE59BD9B4E019ULL);
    for (int i = 0; i < 4; ++i) r->s[i] = splitmix64(&x);
}
static inline uint64_t rng_next(rng_t* r) {   // xoshiro256**
    uint64_t* s = r->s;
    uint64_t result = rotl(s[1] * 5, 7) * 9;
    uint64_t t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t; s[3] = rotl(s[3], 45);
    return result;
}
static inline double rng_unif(rng_t* r) { return (double)(rng_next(r) >> 11) * (1.0 / 9007199254740992.0); }
static inline uint64_t rng_below(rng_t* r, uint64_t n) { return n ? rng_next(r) % n : 0; }

static const char ACGT[4] = {'A', 'C', 'G', 'T'};
static const char acgt[4] = {'a', 'c', 'g', 't'};
static inline int base_code(char c) {
    switch (c) { case 'A': case 'a': return 0; case 'C': case 'c': return 1; case 'G': case 'g': return 2; case 'T': case 't': return 3; default: return 4; }
}

static const int64_t HG38_LENS[24] = {
    248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973, 145138636,
    138394717, 133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345,
    83257441, 80373285, 58617616, 64444167, 46709983, 50818468, 156040895, 57227415};
static const char* HG38_NAMES[24] = {"chr1", "chr2", "chr3", "chr4", "chr5", "chr6", "chr7", "chr8", "chr9", "chr10", "chr11", "chr12",
                                     "chr13", "chr14", "chr15", "chr16", "chr17", "chr18", "chr19", "chr20", "chr21", "chr22", "chrX", "chrY"};

typedef struct {
    int n;
    int64_t lens[64];
    char names[64][16];
    double gc;
    double alu_frac, l1_frac, sat_frac, sd_frac, is_frac;
    int64_t telomere_n, gap_n;
} preset_t;

static int get_preset(const char* name, double scale, preset_t* p) {
    memset(p, 0, sizeof *p);
    if (scale <= 0) scale = 1.0;
    if (strcmp(name, "hg38") == 0) {
        p->n = 24;
        for (int i = 0; i < 24; ++i) { p->lens[i] = (int64_t)(HG38_LENS[i] * scale); if (p->lens[i] < 20000) p->lens[i] = 20000; snprintf(p->names[i], 16, "%s", HG38_NAMES[i]); }
        p->gc = 0.41; p->alu_frac = 0.10; p->l1_frac = 0.17; p->sat_frac = 0.03; p->sd_frac = 0.05;
        p->telomere_n = (int64_t)(10000 * (scale < 1 ? (scale < 0.05 ? 0.05 : scale) : 1)); p->gap_n = (int64_t)(50000 * (scale < 1 ? (scale < 0.05 ? 0.05 : scale) : 1));
        return 0;
    }
    if (strcmp(name, "ecoli") == 0) {
        p->n = 1; p->lens[0] = (int64_t)(4641652 * scale); snprintf(p->names[0], 16, "NC_000913.3");
        p->gc = 0.508; p->is_frac = 0.01;
        return 0;
    }
    if (strcmp(name, "chr8chr12") == 0) {   // config C1: hg38 chr8 + chr12 lengths
        p->n = 2;
        p->lens[0] = (int64_t)(HG38_LENS[7] * scale); p->lens[1] = (int64_t)(HG38_LENS[11] * scale);
        snprintf(p->names[0], 16, "chr8"); snprintf(p->names[1], 16, "chr12");
        p->gc = 0.41; p->alu_frac = 0.10; p->l1_frac = 0.17; p->sat_frac = 0.03; p->sd_frac = 0.05;
        p->telomere_n = 10000; p->gap_n = 50000;
        return 0;
    }
    if (strcmp(name, "small") == 0) {
        p->n = 3; p->lens[0] = (int64_t)(60000 * scale); p->lens[1] = (int64_t)(45000 * scale); p->lens[2] = (int64_t)(30000 * scale);
        snprintf(p->names[0], 16, "ctgA"); snprintf(p->names[1], 16, "ctgB"); snprintf(p->names[2], 16, "ctgC");
        p->gc = 0.41; p->alu_frac = 0.10; p->l1_frac = 0.17; p->sat_frac = 0.03; p->sd_frac = 0.05;
        p->telomere_n = 200; p->gap_n = 500;
        return 0;
    }
    return -1;
}

static inline char rand_base(rng_t* r, double gc) {
    double u = rng_unif(r);
    if (u < gc * 0.5) return 'C';
    if (u < gc) return 'G';
    if (u < gc + (1 - gc) * 0.5) return 'A';
    return 'T';
}

// Write a mutated copy of src[0..n) (optionally reverse-complemented) into dst
// (at most cap bytes). Returns bytes written. Divergence d: 80 % subs, 10 % ins, 10 % del.
static int64_t mutate_copy(rng_t* r, const char* src, int64_t n, int rc, double d, int lower, char* dst, int64_t cap) {
    int64_t o = 0;
    for (int64_t t = 0; t < n && o < cap; ++t) {
        char c = rc ? src[n - 1 - t] : src[t];
        int code = base_code(c);
        if (rc && code < 4) code = 3 - code;
        double u = rng_unif(r);
        if (u < d) {
            double v = rng_unif(r);
            if (v < 0.8) { code = (code + 1 + (int)rng_below(r, 3)) & 3; }
            else if (v < 0.9) { if (o < cap) dst[o++] = lower ? acgt[rng_below(r, 4)] : ACGT[rng_below(r, 4)]; }
            else continue;
        }
        if (o < cap) dst[o++] = code < 4 ? (lower ? acgt[code] : ACGT[code]) : 'N';
    }
    return o;
}

typedef struct {
    const preset_t* p; uint64_t seed; int ci; char* out;
    const char* alu; const char* l1; const char* sat; const char* is_el;
} ctg_job_t;

static void fill_contig(ctg_job_t* J) {
    const preset_t* p = J->p;
    int64_t L = p->lens[J->ci];
    char* s = J->out;
    rng_t r; rng_seed(&r, J->seed, 1000 + (uint64_t)J->ci);
    for (int64_t i = 0; i < L; ++i) s[i] = rand_base(&r, p->gc);
    char* tmp = (char*)malloc(200000);
    // IS elements (ecoli): 1.3 kb, near-identical copies
    if (p->is_frac > 0) {
        int64_t ncopy = (int64_t)(p->is_frac * L / 1300.0);
        for (int64_t c = 0; c < ncopy; ++c) {
            int64_t pos = (int64_t)rng_below(&r, (uint64_t)(L - 1400));
            int64_t w = mutate_copy(&r, J->is_el, 1300, (int)rng_below(&r, 2), 0.002, 0, tmp, 1400);
            memcpy(s + pos, tmp, (size_t)w);
        }
    }
    // Segmental duplications: copy a 10-100 kb segment from elsewhere in this contig, 1-4 % divergence
    if (p->sd_frac > 0) {
        int64_t done = 0, target = (int64_t)(p->sd_frac * L);
        int64_t maxseg = L / 4 < 100000 ? L / 4 : 100000, minseg = maxseg < 10000 ? maxseg / 2 : 10000;
        char* seg = (char*)malloc((size_t)maxseg + 16);
        while (done < target && maxseg > 100) {
            int64_t len = minseg + (int64_t)rng_below(&r, (uint64_t)(maxseg - minseg + 1));
            int64_t a = (int64_t)rng_below(&r, (uint64_t)(L - len)), b = (int64_t)rng_below(&r, (uint64_t)(L - len));
            memcpy(seg, s + a, (size_t)len);
            int64_t w = mutate_copy(&r, seg, len, (int)rng_below(&r, 2), 0.01 + 0.03 * rng_unif(&r), 0, tmp, len < 200000 ? len : 200000);
            memcpy(s + b, tmp, (size_t)w);
            done += len;
        }
        free(seg);
    }
    // L1-like fragments (3'-biased sub-intervals of the 6 kb consensus), 5-20 %
    if (p->l1_frac > 0) {
        int64_t done = 0, target = (int64_t)(p->l1_frac * L);
        while (done < target) {
            int64_t fl = 300 + (int64_t)(5700.0 * rng_unif(&r) * rng_unif(&r));
            int64_t st = 6000 - fl;
            int64_t pos = (int64_t)rng_below(&r, (uint64_t)(L - fl - 600 > 1 ? L - fl - 600 : 1));
            int64_t w = mutate_copy(&r, J->l1 + st, fl, (int)rng_below(&r, 2), 0.05 + 0.15 * rng_unif(&r), 1, tmp, fl + 600);
            if (pos + w > L) w = L - pos;
            memcpy(s + pos, tmp, (size_t)w);
            done += w;
        }
    }
    // Alu-like 300 bp, 10-15 %
    if (p->alu_frac > 0) {
        int64_t ncopy = (int64_t)(p->alu_frac * L / 300.0);
        for (int64_t c = 0; c < ncopy; ++c) {
            int64_t pos = (int64_t)rng_below(&r, (uint64_t)(L - 400 > 1 ? L - 400 : 1));
            int64_t w = mutate_copy(&r, J->alu, 300, (int)rng_below(&r, 2), 0.10 + 0.05 * rng_unif(&r), 1, tmp, 400);
            if (pos + w > L) w = L - pos;
            memcpy(s + pos, tmp, (size_t)w);
        }
    }
    // Satellite array (171 bp monomer, 2-5 % per copy) around the middle
    if (p->sat_frac > 0) {
        int64_t arr = (int64_t)(p->sat_frac * L);
        int64_t pos = L / 2 - arr / 2;
        int64_t o = 0;
        while (o < arr) {
            int64_t w = mutate_copy(&r, J->sat, 171, 0, 0.02 + 0.03 * rng_unif(&r), 1, tmp, 200);
            if (o + w > arr) w = arr - o;
            memcpy(s + pos + o, tmp, (size_t)w);
            o += w;
        }
        // N gap beside the array
        if (p->gap_n > 0 && pos > p->gap_n) memset(s + pos - p->gap_n, 'N', (size_t)p->gap_n);
    }
    if (p->telomere_n > 0 && L > 4 * p->telomere_n) { memset(s, 'N', (size_t)p->telomere_n); memset(s + L - p->telomere_n, 'N', (size_t)p->telomere_n); }
    free(tmp);
}

static void* fill_thread(void* arg) {
    ctg_job_t* jobs = (ctg_job_t*)arg;
    (void)jobs;
    return NULL;
}

typedef struct { ctg_job_t* jobs; int n; int* next; pthread_mutex_t* mu; } pool_t;
static void* pool_worker(void* arg) {
    pool_t* P = (pool_t*)arg;
    for (;;) {
        pthread_mutex_lock(P->mu);
        int i = (*P->next)++;
        pthread_mutex_unlock(P->mu);
        if (i >= P->n) break;
        fill_contig(&P->jobs[i]);
    }
    return NULL;
}

// ---------------------------------------------------------------- C ABI
// Number of contigs and their lengths/names (names: n x 16 bytes).
int sim_genome_layout(const char* preset, double scale, int64_t* lens, char* names16, int max) {
    preset_t p;
    if (get_preset(preset, scale, &p) != 0) return -1;
    for (int i = 0; i < p.n && i < max; ++i) { lens[i] = p.lens[i]; if (names16) memcpy(names16 + 16 * i, p.names[i], 16); }
    return p.n;
}

// Fill buf (sum of lens bytes) with the concatenated contigs.
int sim_genome_fill(const char* preset, double scale, uint64_t seed, char* buf, int nthreads) {
    preset_t p;
    if (get_preset(preset, scale, &p) != 0) return -1;
    rng_t r; rng_seed(&r, seed, 7);
    char alu[300], l1[6000], sat[171], is_el[1300];
    for (int i = 0; i < 300; ++i) alu[i] = rand_base(&r, 0.52);
    for (int i = 0; i < 6000; ++i) l1[i] = rand_base(&r, 0.40);
    for (int i = 0; i < 171; ++i) sat[i] = rand_base(&r, 0.38);
    for (int i = 0; i < 1300; ++i) is_el[i] = rand_base(&r, 0.50);
    ctg_job_t jobs[64];
    int64_t off = 0;
    for (int i = 0; i < p.n; ++i) {
        jobs[i].p = &p; jobs[i].seed = seed; jobs[i].ci = i; jobs[i].out = buf + off;
        jobs[i].alu = alu; jobs[i].l1 = l1; jobs[i].sat = sat; jobs[i].is_el = is_el;
        off += p.lens[i];
    }
    if (nthreads < 1) nthreads = 1;
    if (nthreads > p.n) nthreads = p.n;
    int next = 0; pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    // largest-first (contigs are listed roughly by size already)
    pool_t P = {jobs, p.n, &next, &mu};
    pthread_t th[64];
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, pool_worker, &P);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    (void)fill_thread;
    return 0;
}

// Simulate n reads from a genome given as concatenated contigs.  Output bases
// go to out (capacity cap); offs[n+1] offsets; origin info (4 ints per read:
// contig, start, strand, has_N_run) if non-null.  Returns total bases or -1.
int64_t sim_reads(const char* genome, const int64_t* ctg_lens, int n_ctg, int64_t n_reads, int64_t read_len, uint64_t seed,
                  char* out, int64_t cap, int64_t* offs, int64_t* origin) {
    int64_t* ctg_off = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_ctg + 1));
    ctg_off[0] = 0;
    for (int i = 0; i < n_ctg; ++i) ctg_off[i + 1] = ctg_off[i] + ctg_lens[i];
    int64_t total = ctg_off[n_ctg];
    char* tmpl = (char*)malloc((size_t)read_len + 1);
    int64_t o = 0;
    for (int64_t ri = 0; ri < n_reads; ++ri) {
        rng_t r; rng_seed(&r, seed, 1000000 + (uint64_t)ri);
        int ci = 0; int64_t st = 0; int ok = 0;
        for (int attempt = 0; attempt < 1000 && !ok; ++attempt) {
            int64_t g = (int64_t)rng_below(&r, (uint64_t)total);
            ci = 0; while (ci + 1 < n_ctg && g >= ctg_off[ci + 1]) ++ci;
            int64_t L = ctg_lens[ci];
            if (L <= read_len) continue;
            st = (int64_t)rng_below(&r, (uint64_t)(L - read_len));
            ok = 1;
            const char* src = genome + ctg_off[ci] + st;
            for (int64_t t = 0; t < read_len; ++t) if (base_code(src[t]) == 4) { ok = 0; break; }
        }
        if (!ok) { free(ctg_off); free(tmpl); return -1; }
        int strand = (int)rng_below(&r, 2);
        memcpy(tmpl, genome + ctg_off[ci] + st, (size_t)read_len);
        offs[ri] = o;
        for (int64_t t = 0; t < read_len; ++t) {
            char c = strand ? tmpl[read_len - 1 - t] : tmpl[t];
            int code = base_code(c);
            if (strand) code = 3 - code;
            double u = rng_unif(&r);
            if (u < 0.035) { code = (code + 1 + (int)rng_below(&r, 3)) & 3; }
            else if (u < 0.0575) {
                int ins = rng_unif(&r) < 0.5 ? code : (int)rng_below(&r, 4);
                if (o < cap) out[o++] = ACGT[ins];
            } else if (u < 0.08) continue;
            if (o < cap) out[o++] = ACGT[code];
        }
        int has_n = 0;
        if (rng_unif(&r) < 0.0005 && o - offs[ri] > 40) {
            int64_t len = o - offs[ri];
            int64_t p0 = offs[ri] + (int64_t)rng_below(&r, (uint64_t)(len - 20));
            memset(out + p0, 'N', 20);
            has_n = 1;
        }
        if (origin) { origin[4 * ri] = ci; origin[4 * ri + 1] = st; origin[4 * ri + 2] = strand; origin[4 * ri + 3] = has_n; }
        if (o >= cap) { free(ctg_off); free(tmpl); return -1; }
    }
    offs[n_reads] = o;
    free(ctg_off); free(tmpl);
    return o;
}

// ---------------------------------------------------------------- CLI
#ifdef SIMGEN_MAIN
static int write_fasta_rec(FILE* f, const char* name, const char* s, int64_t n) {
    fprintf(f, ">%s\n", name);
    for (int64_t i = 0; i < n; i += 80) { int64_t w = n - i < 80 ? n - i : 80; fwrite(s + i, 1, (size_t)w, f); fputc('\n', f); }
    return 0;
}
static char* read_fasta_all(const char* path, int64_t* lens, int* n, int max, int64_t* tot) {
    FILE* f = fopen(path, "rb"); if (!f) return NULL;
    fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
    char* raw = (char*)malloc((size_t)sz + 1); if (fread(raw, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); return NULL; } fclose(f);
    char* seq = (char*)malloc((size_t)sz + 1); int64_t o = 0; *n = -1;
    for (long i = 0; i < sz;) {
        long e = i; while (e < sz && raw[e] != '\n') ++e;
        if (raw[i] == '>') { if (*n + 1 >= max) break; ++*n; lens[*n] = 0; }
        else if (*n >= 0) { for (long t = i; t < e; ++t) if (raw[t] != '\r') { seq[o++] = raw[t]; lens[*n]++; } }
        i = e + 1;
    }
    *n += 1; *tot = o; free(raw); return seq;
}
int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: simgen genome <preset> <scale> <seed> <out.fa> [threads]\n       simgen reads <ref.fa> <n> <len> <seed> <out.fa>\n"); return 2; }
    if (strcmp(argv[1], "genome") == 0 && argc >= 6) {
        int64_t lens[64]; char names[64 * 16];
        int n = sim_genome_layout(argv[2], atof(argv[3]), lens, names, 64);
        if (n < 0) { fprintf(stderr, "unknown preset\n"); return 1; }
        int64_t tot = 0; for (int i = 0; i < n; ++i) tot += lens[i];
        char* buf = (char*)malloc((size_t)tot);
        sim_genome_fill(argv[2], atof(argv[3]), strtoull(argv[4], NULL, 10), buf, argc > 6 ? atoi(argv[6]) : 8);
        FILE* f = fopen(argv[5], "wb"); int64_t off = 0;
        for (int i = 0; i < n; ++i) { write_fasta_rec(f, names + 16 * i, buf + off, lens[i]); off += lens[i]; }
        fclose(f); free(buf); return 0;
    }
    if (strcmp(argv[1], "reads") == 0 && argc >= 7) {
        int64_t lens[4096]; int n; int64_t tot;
        char* g = read_fasta_all(argv[2], lens, &n, 4096, &tot);
        if (!g) { fprintf(stderr, "cannot read %s\n", argv[2]); return 1; }
        int64_t nr = atoll(argv[3]), rl = atoll(argv[4]);
        int64_t cap = nr * rl * 2 + 1024;
        char* out = (char*)malloc((size_t)cap); int64_t* offs = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nr + 1));
        if (sim_reads(g, lens, n, nr, rl, strtoull(argv[5], NULL, 10), out, cap, offs, NULL) < 0) { fprintf(stderr, "simulation failed\n"); return 1; }
        FILE* f = fopen(argv[6], "wb"); char nm[32];
        for (int64_t i = 0; i < nr; ++i) { snprintf(nm, sizeof nm, "r%lld", (long long)i); write_fasta_rec(f, nm, out + offs[i], offs[i + 1] - offs[i]); }
        fclose(f); return 0;
    }
    fprintf(stderr, "bad arguments\n"); return 2;
}
#endif
