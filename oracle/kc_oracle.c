/*
 * kc_oracle.c — CPU ORACLE for the k-mer count path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (libkc_hip.so, the
 * kmer-counter CLI, kmer-counter_amd/) links, loads or calls this file. It is
 * used by tests/ as the checker, by __graft_entry__.smoke() as the checker and
 * by bench.py's cpu_baseline leg as the timed CPU port ("refcpu").
 *
 * It restates, in plain C, the reference's count path:
 *   - FASTQFileReader::FASTQFileReader / readData / isComplete
 *     (FASTQFileReader.cpp:18-41, 49-89, 91-93) and InputFileHandler::read
 *     (InputFileHandler.cpp:82-95) over an in-memory file, with libstdc++
 *     std::getline / tellg semantics;
 *   - KMerCounter::GetChunkSize (KMerCounter.cpp:193-212);
 *   - bitEncode (GPUHandler.cu:10-111), checkBit/read64bits (:113-127),
 *     extractKMers (:129-233), calculateOutputSize (:235-245),
 *     CheckEquals/reduceKMers (:329-360) — "ref-structured" form, same buffer
 *     layout (u16 2L header + MSB-first words in place at stride L, N-mask
 *     filter at stride L, per-read output sections with zeroed holes);
 *   - the same semantics as a direct per-window formula ("spec" form,
 *     SURVEY Appendix A), used to cross-check the ref-structured form;
 *   - KMerCounter::dispatchWork's hash aggregation (KMerCounter.cpp:61-82) with
 *     a sharded-lock table in place of TBB concurrent_hash_map, and the
 *     SortedKMerFile record format (SortedKMerFile.cpp, KMerFileMerger.cpp:98-135).
 *
 * Parity pinning: the reader, chunking, merge and
 * printer restatements are checked against the reference's own C++ sources
 * compiled unmodified into oracle/_ref/ (oracle/ref/Makefile). GPUHandler.cu
 * itself needs nvcc, the CUDA headers and thrust, none of which exist here, so
 * the window/encode semantics are pinned only by the two restatements below
 * agreeing with each other and with SURVEY Appendix A.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define O_MAXW 4

/* ------------------------------------------------------------------------- */
/* helpers                                                                   */
/* ------------------------------------------------------------------------- */

static int o_words(int64_t k) { return (int)((k + 31) / 32); }

/* GPUHandler.cu:181-186,210-213: the last key word is masked to k%32 bases only
 * when ceil(k/4) < 8W. */
static int o_masks_last_word(int64_t k) { return ((k + 3) / 4) < 8 * (int64_t)o_words(k); }

static unsigned o_code(unsigned char c) {
    switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    default: return 3; /* GPUHandler.cu:79-87: every other byte encodes as 3 */
    }
}

static int o_bad(unsigned char c) { return !(c == 'A' || c == 'C' || c == 'G' || c == 'T'); }

static uint64_t o_ld64(const unsigned char* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

static void o_st64(unsigned char* p, uint64_t v) { memcpy(p, &v, 8); }

static int o_cmp_words(const uint64_t* a, const uint64_t* b, int W) {
    for (int j = 0; j < W; j++) {
        if (a[j] < b[j]) return -1;
        if (a[j] > b[j]) return 1;
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* KMerCounter::GetChunkSize (KMerCounter.cpp:193-212)                        */
/* ------------------------------------------------------------------------- */

int64_t oracle_chunk_size(int64_t line_length, int64_t kmer_length, int64_t gpu_memory_limit) {
    int64_t key_bytes = (kmer_length + 3) / 4;
    int64_t record_bytes = ((key_bytes + 7) / 8 + 1) * 8; /* words + 1 "count" word */
    int64_t per_read = record_bytes * (line_length - kmer_length + 1);
    if (per_read - 1 == 0) return 0;
    int64_t reads = (gpu_memory_limit - line_length) / (per_read - 1);
    return line_length * reads;
}

/* ------------------------------------------------------------------------- */
/* FASTQ chunk reader over an in-memory file (FASTQFileReader.cpp)           */
/* ------------------------------------------------------------------------- */

typedef struct o_stream {
    const char* p;
    int64_t n;
    int64_t pos;
    int eof, fail;
} o_stream;

/* std::getline(istream&, string&) as implemented by libstdc++: a failed sentry
 * (stream not good) leaves the string untouched; otherwise the string is
 * cleared and bytes up to '\n' are extracted ('\n' consumed, not stored);
 * running into the end sets eof, and fail too if nothing was extracted. */
static void o_getline(o_stream* st, const char** s, int64_t* len) {
    if (st->eof || st->fail) return;
    const char* start = st->p + st->pos;
    const char* nl = (const char*)memchr(start, '\n', (size_t)(st->n - st->pos));
    if (nl) {
        *s = start;
        *len = nl - start;
        st->pos = (nl - st->p) + 1;
        return;
    }
    *s = start;
    *len = st->n - st->pos;
    st->pos = st->n;
    st->eof = 1;
    if (*len == 0) st->fail = 1;
}

/* istream::tellg: its sentry sets failbit on a stream that is not good, and
 * then -1 is returned. */
static int64_t o_tellg(o_stream* st) {
    if (st->eof || st->fail) {
        st->fail = 1;
        return -1;
    }
    return st->pos;
}

typedef struct oracle_reader {
    o_stream st;
    int64_t file_size;
    int64_t line_length;
    int done;
} oracle_reader;

/* FASTQFileReader ctor (FASTQFileReader.cpp:18-41): L = length of line 2. */
oracle_reader* oracle_reader_new(const char* data, int64_t n) {
    oracle_reader* r = (oracle_reader*)calloc(1, sizeof(*r));
    r->st.p = data;
    r->st.n = n;
    r->file_size = n;
    const char* s = NULL;
    int64_t len = 0, len2 = 0;
    o_getline(&r->st, &s, &len);
    o_getline(&r->st, &s, &len2);
    r->line_length = len2;
    /* seekg(0): C++11 clears eofbit first; a failed stream does not seek. */
    r->st.eof = 0;
    if (!r->st.fail) r->st.pos = 0;
    return r;
}

int64_t oracle_reader_line_length(const oracle_reader* r) { return r->line_length; }
int oracle_reader_done(const oracle_reader* r) { return r->done; }
void oracle_reader_free(oracle_reader* r) { free(r); }

/* One call of InputFileHandler::read -> FASTQFileReader::readData for a single
 * file (InputFileHandler.cpp:82-95, FASTQFileReader.cpp:49-93). The sequence
 * lines are concatenated without separators into dst (capacity chunk_size);
 * returns the chunk's byte size. Sets done when the handler would pop the
 * file. */
int64_t oracle_reader_next(oracle_reader* r, int64_t chunk_size, char* dst) {
    if (r->done) return -1;
    int64_t off = 0;
    const char* temp = "";
    int64_t temp_len = 0;
    const char* line = "";
    int64_t line_len = 0;
    o_getline(&r->st, &temp, &temp_len);
    o_getline(&r->st, &line, &line_len);
    while (line_len != 0 && off + temp_len < chunk_size) {
        if (line[0] == '+') {
            /* the else branch at FASTQFileReader.cpp:72-74 is unreachable: its
               condition repeats the loop condition */
            memcpy(dst + off, temp, (size_t)temp_len);
            off += temp_len;
            o_getline(&r->st, &temp, &temp_len);
            o_getline(&r->st, &line, &line_len);
        } else {
            temp = line;
            temp_len = line_len;
            o_getline(&r->st, &line, &line_len);
        }
    }
    if (off < chunk_size) dst[off] = '\0';
    int64_t pos = o_tellg(&r->st);
    if (pos + r->line_length > r->file_size || off == 0) r->done = 1;
    return off;
}

/* ------------------------------------------------------------------------- */
/* spec form: one window -> key words                    */
/* ------------------------------------------------------------------------- */

static void o_spec_key(const unsigned char* s, int64_t L, int64_t k, int64_t p, uint64_t* out) {
    int W = o_words(k);
    for (int j = 0; j < W; j++) {
        uint64_t w = 0;
        for (int b = 0; b < 32; b++) {
            int64_t i = p + 32 * (int64_t)j + b;
            uint64_t c = (i < L) ? o_code(s[i]) : 0; /* past the read end: 0 */
            w |= c << (62 - 2 * b);
        }
        out[j] = w;
    }
    if (o_masks_last_word(k)) {
        int keep = (int)(k % 32);
        out[W - 1] &= ~0ull << (64 - 2 * keep);
    }
}

/* ------------------------------------------------------------------------- */
/* accumulator: a growable array of keys (sort + reduce at the end)          */
/* ------------------------------------------------------------------------- */

typedef struct oracle_acc {
    int64_t k;
    int W;
    uint64_t* keys; /* n * W words */
    uint32_t* cnts; /* count per entry (reduced records carry counts > 1) */
    int64_t n, cap;
    int hole; /* a zeroed hole record reached the hash (key 0^W, count 0) */
    uint64_t windows, valid;
} oracle_acc;

oracle_acc* oracle_acc_new(int64_t k) {
    if (k < 1 || k > 32 * O_MAXW) return NULL;
    oracle_acc* a = (oracle_acc*)calloc(1, sizeof(*a));
    a->k = k;
    a->W = o_words(k);
    return a;
}

void oracle_acc_free(oracle_acc* a) {
    if (!a) return;
    free(a->keys);
    free(a->cnts);
    free(a);
}

static void o_acc_push(oracle_acc* a, const uint64_t* key, uint32_t cnt) {
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 1024;
        a->keys = (uint64_t*)realloc(a->keys, (size_t)a->cap * a->W * 8);
        a->cnts = (uint32_t*)realloc(a->cnts, (size_t)a->cap * 4);
    }
    memcpy(a->keys + a->n * a->W, key, (size_t)a->W * 8);
    a->cnts[a->n] = cnt;
    a->n++;
}

/* spec form of processKMers + hash insert for one chunk. */
void oracle_acc_add_chunk_spec(oracle_acc* a, const char* chunk, int64_t size, int64_t L) {
    int64_t k = a->k;
    if (L < k || L <= 0) return;
    int64_t n = size / L;
    uint64_t key[O_MAXW];
    for (int64_t r = 0; r < n; r++) {
        const unsigned char* s = (const unsigned char*)chunk + r * L;
        int64_t last_bad = -1;
        for (int64_t i = 0; i < k - 1; i++)
            if (o_bad(s[i])) last_bad = i;
        for (int64_t p = 0; p + k <= L; p++) {
            if (o_bad(s[p + k - 1])) last_bad = p + k - 1;
            a->windows++;
            if (last_bad >= p) {
                a->hole = 1;
                continue;
            }
            a->valid++;
            o_spec_key(s, L, k, p, key);
            o_acc_push(a, key, 1);
        }
    }
}

/* ------------------------------------------------------------------------- */
/* ref-structured form of processKMers (GPUHandler.cu:397-466)               */
/* ------------------------------------------------------------------------- */

/* bitEncode for the read at byte offset `base` of `buf` (GPUHandler.cu:10-111):
 * in place, [u16 2L][ceil(L/32) words], the trailing word left-aligned, plus
 * the N-mask (1 = not ACGT) MSB-first at the same offset of `filt`. Defined
 * for L % 32 != 0 (for L % 32 == 0 the reference shifts by 64: undefined). */
static void o_ref_encode(unsigned char* buf, unsigned char* filt, int64_t base, int64_t L) {
    uint64_t word = 0, mask = 0;
    for (int64_t i = 0; i < L; i++) {
        if (i > 0 && i % 32 == 0) {
            o_st64(buf + base + 2 + 8 * (i / 32 - 1), word);
            word = 0;
        }
        if (i > 0 && i % 64 == 0) {
            o_st64(filt + base + 8 * (i / 64 - 1), mask);
            mask = 0;
        }
        unsigned char c = buf[base + i];
        word = (word << 2) | o_code(c);
        mask = (mask << 1) | (uint64_t)o_bad(c);
    }
    uint16_t hdr = (uint16_t)(2 * L);
    memcpy(buf + base, &hdr, 2);
    if (L % 64 > 0) {
        word <<= 2 * (32 - L % 32);
        o_st64(buf + base + 2 + 8 * (L / 32), word);
        mask <<= 64 - L % 64;
        o_st64(filt + base + 8 * (L / 64), mask);
    }
}

/* extractKMers for one read (GPUHandler.cu:129-233): valid windows written in
 * order from the start of the read's output section; the rest stays zero. */
static void o_ref_extract(const unsigned char* buf, const unsigned char* filt, int64_t base, int64_t k,
                          unsigned char* section) {
    uint16_t hdr;
    memcpy(&hdr, buf + base, 2);
    int64_t len = hdr / 2;
    const unsigned char* enc = buf + base + 2;
    int W = o_words(k);
    int64_t key_bytes = (k + 3) / 4;
    int last_mask = o_masks_last_word(k);
    int rshift = (int)(32 - k % 32) * 2;
    int64_t run = 0, out = 0;
    for (int64_t i = 0; i < len; i++) {
        uint64_t f = o_ld64(filt + base + 8 * (i / 64));
        int bad = (int)((f >> (63 - (i % 64))) & 1);
        if (bad) {
            run = 0;
            continue;
        }
        if (++run < k) continue;
        int64_t p = i - k + 1;
        int shift = (int)(p % 32) * 2;
        int64_t first = (p / 32) * 8;
        for (int j = 0; j < W; j++) {
            int64_t x = first + 8 * j;
            uint64_t v = o_ld64(enc + x);
            if (shift > 0) {
                v <<= shift;
                if ((x + 8) * 4 < len) v |= o_ld64(enc + x + 8) >> (64 - shift);
            }
            if (j == W - 1 && last_mask && x + 8 > first + key_bytes) v = (v >> rshift) << rshift;
            o_st64(section + out, v);
            out += 8;
        }
        uint32_t one = 1;
        memcpy(section + out, &one, 4);
        out += 4;
        run--;
    }
}

/* reduceKMers (GPUHandler.cu:340-360): fold runs of adjacent equal keys. */
static int64_t o_ref_reduce(unsigned char* recs, int64_t bytes, int rs) {
    if (bytes <= 0) return 0;
    int64_t keep = 0;
    for (int64_t i = rs; i < bytes; i += rs) {
        if (memcmp(recs + keep, recs + i, (size_t)(rs - 4)) == 0) {
            uint32_t a, b;
            memcpy(&a, recs + keep + rs - 4, 4);
            memcpy(&b, recs + i + rs - 4, 4);
            a += b;
            memcpy(recs + keep + rs - 4, &a, 4);
        } else {
            keep += rs;
            if (keep != i) memmove(recs + keep, recs + i, (size_t)rs);
        }
    }
    return keep + rs;
}

/* Per-worker buffers of processKMers' data path, allocated once and reused
 * per chunk like the reference's per-stream buffers (PrepareGPU allocates
 * h_output once; processKMers memsets it per chunk, GPUHandler.cu:406,490). */
typedef struct o_ws {
    unsigned char *buf, *filt, *recs;
    size_t cap_buf, cap_recs;
} o_ws;

static void o_ws_fit(o_ws* w, size_t buf, size_t recs) {
    if (buf > w->cap_buf) {
        free(w->buf);
        free(w->filt);
        w->buf = (unsigned char*)malloc(buf);
        w->filt = (unsigned char*)malloc(buf);
        w->cap_buf = buf;
    }
    if (recs > w->cap_recs) {
        free(w->recs);
        w->recs = (unsigned char*)malloc(recs);
        w->cap_recs = recs;
    }
}

static void o_ws_free(o_ws* w) {
    free(w->buf);
    free(w->filt);
    free(w->recs);
    memset(w, 0, sizeof(*w));
}

/* Runs processKMers' data path for one chunk; the reduced records are left at
 * the start of w->recs and their byte length is returned. */
static int64_t o_ref_process_chunk_ws(o_ws* w, const char* chunk, int64_t size, int64_t L, int64_t k) {
    int W = o_words(k);
    int rs = 8 * W + 4;
    int64_t n = size / L;
    int64_t per_read = (L - k + 1) * rs;
    o_ws_fit(w, (size_t)size + 64, (size_t)(n * per_read) + 1);
    memcpy(w->buf, chunk, (size_t)size);
    memset(w->buf + size, 0, 64);
    memset(w->filt, 0, (size_t)size + 64);
    memset(w->recs, 0, (size_t)(n * per_read));
    for (int64_t r = 0; r < n; r++) o_ref_encode(w->buf, w->filt, r * L, L);
    for (int64_t r = 0; r < n; r++) o_ref_extract(w->buf, w->filt, r * L, k, w->recs + r * per_read);
    return o_ref_reduce(w->recs, n * per_read, rs);
}

static int64_t o_ref_process_chunk(const char* chunk, int64_t size, int64_t L, int64_t k, unsigned char** out) {
    o_ws w;
    memset(&w, 0, sizeof(w));
    int64_t bytes = o_ref_process_chunk_ws(&w, chunk, size, L, k);
    *out = w.recs;
    w.recs = NULL;
    o_ws_free(&w);
    return bytes;
}

void oracle_acc_add_chunk_ref(oracle_acc* a, const char* chunk, int64_t size, int64_t L) {
    int64_t k = a->k;
    if (L < k || L <= 0 || size < L) return;
    int W = a->W, rs = 8 * W + 4;
    unsigned char* recs = NULL;
    int64_t bytes = o_ref_process_chunk(chunk, size, L, k, &recs);
    uint64_t key[O_MAXW];
    for (int64_t off = 0; off < bytes; off += rs) {
        uint32_t c;
        memcpy(key, recs + off, (size_t)W * 8);
        memcpy(&c, recs + off + 8 * W, 4);
        o_acc_push(a, key, c);
    }
    free(recs);
}

/* ------------------------------------------------------------------------- */
/* finish: sort, fold equal keys (u32 sums), SortedKMerFile bytes            */
/* ------------------------------------------------------------------------- */

static int g_sort_w; /* qsort has no context argument */
static int o_qcmp(const void* x, const void* y) {
    return o_cmp_words((const uint64_t*)x, (const uint64_t*)y, g_sort_w);
}

static pthread_mutex_t g_sort_mu = PTHREAD_MUTEX_INITIALIZER;

/* Sorts and folds the accumulated entries. Returns the number of output
 * records and stores the SortedKMerFile bytes in *out (malloc; free with
 * oracle_free). The hole flag is folded in as a key-0 record with count 0,
 * exactly what a zeroed hole record does when it reaches the hash in the
 * reference (GPUHandler.cu:466 -> KMerCounter.cpp:70). The accumulator is
 * emptied. */
int64_t oracle_acc_finish(oracle_acc* a, unsigned char** out) {
    int W = a->W, rs = 8 * W + 4;
    if (a->hole) {
        uint64_t zero[O_MAXW] = {0, 0, 0, 0};
        o_acc_push(a, zero, 0);
        a->hole = 0;
    }
    int64_t n = a->n;
    size_t ent = (size_t)W * 8 + 8;
    unsigned char* tmp = (unsigned char*)malloc(ent * (size_t)(n ? n : 1));
    for (int64_t i = 0; i < n; i++) {
        memcpy(tmp + i * ent, a->keys + i * W, (size_t)W * 8);
        uint64_t c = a->cnts[i];
        memcpy(tmp + i * ent + W * 8, &c, 8);
    }
    pthread_mutex_lock(&g_sort_mu);
    g_sort_w = W;
    qsort(tmp, (size_t)n, ent, o_qcmp);
    pthread_mutex_unlock(&g_sort_mu);
    unsigned char* res = (unsigned char*)malloc((size_t)(n * rs) + 1);
    int64_t m = 0;
    for (int64_t i = 0; i < n; i++) {
        const unsigned char* e = tmp + i * ent;
        uint64_t c64;
        memcpy(&c64, e + W * 8, 8);
        uint32_t c = (uint32_t)c64;
        if (m > 0 && memcmp(res + (m - 1) * rs, e, (size_t)W * 8) == 0) {
            uint32_t prev;
            memcpy(&prev, res + (m - 1) * rs + W * 8, 4);
            prev += c; /* uint32 wrap, as the reference's counts */
            memcpy(res + (m - 1) * rs + W * 8, &prev, 4);
        } else {
            memcpy(res + m * rs, e, (size_t)W * 8);
            memcpy(res + m * rs + W * 8, &c, 4);
            m++;
        }
    }
    free(tmp);
    a->n = 0;
    *out = res;
    return m;
}

uint64_t oracle_acc_windows(const oracle_acc* a) { return a->windows; }
uint64_t oracle_acc_valid(const oracle_acc* a) { return a->valid; }

/* ------------------------------------------------------------------------- */
/* refcpu: the reference pipeline on the CPU, multi-threaded                 */
/*   main thread: chunker (FASTQFileReader::readData)                        */
/*   T workers:   processKMers data path (ref-structured) + hash insert      */
/*   hash:        sharded locks (TBB concurrent_hash_map stand-in)           */
/* ------------------------------------------------------------------------- */

#define O_SHARDS 1024

typedef struct o_shard {
    pthread_mutex_t mu;
    uint64_t* keys; /* cap * W */
    uint32_t* cnts;
    uint8_t* used;
    int64_t cap, n;
} o_shard;

typedef struct o_table {
    int W;
    o_shard sh[O_SHARDS];
} o_table;

static uint64_t o_mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

static uint64_t o_hash_key(const uint64_t* k, int W) {
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (int j = 0; j < W; j++) h = o_mix64(h ^ k[j]) + (uint64_t)j;
    return h;
}

static void o_shard_grow(o_shard* s, int W) {
    int64_t ncap = s->cap ? s->cap * 2 : 1024;
    uint64_t* nk = (uint64_t*)malloc((size_t)ncap * W * 8);
    uint32_t* nc = (uint32_t*)malloc((size_t)ncap * 4);
    uint8_t* nu = (uint8_t*)calloc((size_t)ncap, 1);
    for (int64_t i = 0; i < s->cap; i++) {
        if (!s->used[i]) continue;
        const uint64_t* key = s->keys + i * W;
        uint64_t h = (o_hash_key(key, W) >> 10) & (uint64_t)(ncap - 1);
        while (nu[h]) h = (h + 1) & (uint64_t)(ncap - 1);
        nu[h] = 1;
        memcpy(nk + h * W, key, (size_t)W * 8);
        nc[h] = s->cnts[i];
    }
    free(s->keys);
    free(s->cnts);
    free(s->used);
    s->keys = nk;
    s->cnts = nc;
    s->used = nu;
    s->cap = ncap;
}

static void o_table_add(o_table* t, const uint64_t* key, uint32_t cnt) {
    int W = t->W;
    uint64_t h = o_hash_key(key, W);
    o_shard* s = &t->sh[h & (O_SHARDS - 1)];
    pthread_mutex_lock(&s->mu);
    if (2 * (s->n + 1) > s->cap) o_shard_grow(s, W);
    uint64_t i = (h >> 10) & (uint64_t)(s->cap - 1);
    for (;;) {
        if (!s->used[i]) {
            s->used[i] = 1;
            memcpy(s->keys + i * W, key, (size_t)W * 8);
            s->cnts[i] = cnt; /* emplace (KMerCounter.cpp:70-72) */
            s->n++;
            break;
        }
        if (memcmp(s->keys + i * W, key, (size_t)W * 8) == 0) {
            s->cnts[i] += cnt; /* acc->second += count (KMerCounter.cpp:75) */
            break;
        }
        i = (i + 1) & (uint64_t)(s->cap - 1);
    }
    pthread_mutex_unlock(&s->mu);
}

typedef struct o_job {
    char* data;
    int64_t size, L;
    struct o_job* next;
} o_job;

typedef struct o_pool {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    o_job* head;
    o_job* tail;
    int closed;
    int64_t queued; /* bound on chunks in flight, like the 8-stream pool */
    pthread_cond_t space;
    o_table* table;
    int64_t k;
} o_pool;

static void* o_worker(void* arg) {
    o_pool* pl = (o_pool*)arg;
    int W = o_words(pl->k), rs = 8 * W + 4;
    o_ws ws;
    memset(&ws, 0, sizeof(ws));
    for (;;) {
        pthread_mutex_lock(&pl->mu);
        while (!pl->head && !pl->closed) pthread_cond_wait(&pl->cv, &pl->mu);
        o_job* j = pl->head;
        if (j) {
            pl->head = j->next;
            if (!pl->head) pl->tail = NULL;
            pl->queued--;
            pthread_cond_signal(&pl->space);
        }
        pthread_mutex_unlock(&pl->mu);
        if (!j) break;
        int64_t bytes = o_ref_process_chunk_ws(&ws, j->data, j->size, j->L, pl->k);
        const unsigned char* recs = ws.recs;
        uint64_t key[O_MAXW];
        for (int64_t off = 0; off < bytes; off += rs) {
            uint32_t c;
            memcpy(key, recs + off, (size_t)W * 8);
            memcpy(&c, recs + off + 8 * W, 4);
            o_table_add(pl->table, key, c);
        }
        free(j->data);
        free(j);
    }
    o_ws_free(&ws);
    return NULL;
}

int64_t oracle_refcpu_run(const char* fastq, int64_t n_bytes, int64_t k, int64_t gpu_memory_limit, int threads,
                          unsigned char** out, uint64_t* windows);

/* Sort of the dumped (key words, u64 count) entries by key: one split by the
 * top 8 bits of word 0 into 256 groups, each group qsorted by one of `threads`
 * workers (the order is the same as one qsort of the whole array; keys are
 * distinct here). Replaces *buf with the sorted copy. */
typedef struct o_psort {
    unsigned char* base;
    const int64_t* start; /* 257 group bounds */
    size_t ent;
    int next; /* next group to take (under mu) */
    pthread_mutex_t mu;
} o_psort;

static void* o_psort_worker(void* arg) {
    o_psort* p = (o_psort*)arg;
    for (;;) {
        pthread_mutex_lock(&p->mu);
        int g = p->next++;
        pthread_mutex_unlock(&p->mu);
        if (g >= 256) break;
        int64_t n = p->start[g + 1] - p->start[g];
        if (n > 1) qsort(p->base + (size_t)p->start[g] * p->ent, (size_t)n, p->ent, o_qcmp);
    }
    return NULL;
}

static void o_par_sort(unsigned char** buf, int64_t m, int W, int threads) {
    size_t ent = (size_t)W * 8 + 8;
    int64_t start[257] = {0}, pos[256];
    for (int64_t i = 0; i < m; i++) start[1 + (o_ld64(*buf + (size_t)i * ent) >> 56)]++;
    for (int g = 0; g < 256; g++) start[g + 1] += start[g];
    memcpy(pos, start, sizeof(pos));
    unsigned char* dst = (unsigned char*)malloc(ent * (size_t)(m ? m : 1));
    for (int64_t i = 0; i < m; i++) {
        const unsigned char* e = *buf + (size_t)i * ent;
        memcpy(dst + (size_t)pos[o_ld64(e) >> 56]++ * ent, e, ent);
    }
    free(*buf);
    *buf = dst;
    pthread_mutex_lock(&g_sort_mu);
    g_sort_w = W;
    o_psort p;
    p.base = dst;
    p.start = start;
    p.ent = ent;
    p.next = 0;
    pthread_mutex_init(&p.mu, NULL);
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, o_psort_worker, &p);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    free(th);
    pthread_mutex_destroy(&p.mu);
    pthread_mutex_unlock(&g_sort_mu);
}

/* Runs the whole reference count path over one in-memory FASTQ file with
 * `threads` workers. Writes the sorted SortedKMerFile bytes into *out (malloc;
 * caller frees with oracle_free) and returns the record count; *windows gets
 * the number of k-mer windows processed. */
int64_t oracle_refcpu_count(const char* fastq, int64_t n_bytes, int64_t k, int64_t gpu_memory_limit, int threads,
                            unsigned char** out, uint64_t* windows) {
    return oracle_refcpu_run(fastq, n_bytes, k, gpu_memory_limit, threads, out, windows);
}

/* out == NULL: stop once the hash table is complete (the reference's work
 * before DumpResults, which writes in hash order) and return the number of
 * distinct keys; used to time the CPU baseline. */
int64_t oracle_refcpu_run(const char* fastq, int64_t n_bytes, int64_t k, int64_t gpu_memory_limit, int threads,
                          unsigned char** out, uint64_t* windows) {
    if (k < 1 || k > 32 * O_MAXW || threads < 1) return -1;
    int W = o_words(k), rs = 8 * W + 4;
    o_table* t = (o_table*)calloc(1, sizeof(*t));
    t->W = W;
    for (int i = 0; i < O_SHARDS; i++) pthread_mutex_init(&t->sh[i].mu, NULL);
    o_pool pl;
    memset(&pl, 0, sizeof(pl));
    pthread_mutex_init(&pl.mu, NULL);
    pthread_cond_init(&pl.cv, NULL);
    pthread_cond_init(&pl.space, NULL);
    pl.table = t;
    pl.k = k;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, o_worker, &pl);

    oracle_reader* rd = oracle_reader_new(fastq, n_bytes);
    int64_t L = rd->line_length;
    int64_t chunk = oracle_chunk_size(L, k, gpu_memory_limit);
    uint64_t nwin = 0;
    if (L >= k && chunk > L) {
        while (!rd->done) {
            char* buf = (char*)malloc((size_t)chunk + 1);
            int64_t sz = oracle_reader_next(rd, chunk, buf);
            if (sz <= 0 || sz < L) {
                free(buf);
                continue;
            }
            nwin += (uint64_t)(sz / L) * (uint64_t)(L - k + 1);
            o_job* j = (o_job*)malloc(sizeof(*j));
            j->data = buf;
            j->size = sz;
            j->L = L;
            j->next = NULL;
            pthread_mutex_lock(&pl.mu);
            while (pl.queued >= 2 * threads) pthread_cond_wait(&pl.space, &pl.mu);
            if (pl.tail)
                pl.tail->next = j;
            else
                pl.head = j;
            pl.tail = j;
            pl.queued++;
            pthread_cond_signal(&pl.cv);
            pthread_mutex_unlock(&pl.mu);
        }
    }
    oracle_reader_free(rd);
    pthread_mutex_lock(&pl.mu);
    pl.closed = 1;
    pthread_cond_broadcast(&pl.cv);
    pthread_mutex_unlock(&pl.mu);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    free(th);

    /* dump: gather entries and sort by key words */
    int64_t total = 0;
    for (int i = 0; i < O_SHARDS; i++) total += t->sh[i].n;
    if (!out) {
        for (int i = 0; i < O_SHARDS; i++) {
            free(t->sh[i].keys);
            free(t->sh[i].cnts);
            free(t->sh[i].used);
            pthread_mutex_destroy(&t->sh[i].mu);
        }
        free(t);
        if (windows) *windows = nwin;
        return total;
    }
    size_t ent = (size_t)W * 8 + 8;
    unsigned char* tmp = (unsigned char*)malloc(ent * (size_t)(total ? total : 1));
    int64_t m = 0;
    for (int i = 0; i < O_SHARDS; i++) {
        o_shard* s = &t->sh[i];
        for (int64_t j = 0; j < s->cap; j++) {
            if (!s->used[j]) continue;
            memcpy(tmp + m * ent, s->keys + j * W, (size_t)W * 8);
            uint64_t c = s->cnts[j];
            memcpy(tmp + m * ent + W * 8, &c, 8);
            m++;
        }
        free(s->keys);
        free(s->cnts);
        free(s->used);
        pthread_mutex_destroy(&s->mu);
    }
    free(t);
    o_par_sort(&tmp, m, W, threads);
    unsigned char* res = (unsigned char*)malloc((size_t)(m * rs) + 1);
    for (int64_t i = 0; i < m; i++) {
        memcpy(res + i * rs, tmp + i * ent, (size_t)W * 8);
        uint64_t c;
        memcpy(&c, tmp + i * ent + W * 8, 8);
        uint32_t c32 = (uint32_t)c;
        memcpy(res + i * rs + W * 8, &c32, 4);
    }
    free(tmp);
    *out = res;
    if (windows) *windows = nwin;
    return m;
}

void oracle_free(void* p) { free(p); }

/* ------------------------------------------------------------------------- */
/* whole-file convenience: reader + chunks + accumulator                      */
/* ------------------------------------------------------------------------- */

/* mode 0 = spec form, 1 = ref-structured form. Returns records (sorted bytes
 * in *out, caller frees with oracle_free), or -1 on bad arguments. */
int64_t oracle_count_fastq(const char* fastq, int64_t n_bytes, int64_t k, int64_t gpu_memory_limit, int mode,
                           unsigned char** out) {
    oracle_acc* a = oracle_acc_new(k);
    if (!a) return -1;
    oracle_reader* rd = oracle_reader_new(fastq, n_bytes);
    int64_t L = rd->line_length;
    int64_t chunk = oracle_chunk_size(L, k, gpu_memory_limit);
    if (L >= k && chunk > L) {
        char* buf = (char*)malloc((size_t)chunk + 1);
        while (!rd->done) {
            int64_t sz = oracle_reader_next(rd, chunk, buf);
            if (sz <= 0 || sz < L) continue;
            if (mode == 1)
                oracle_acc_add_chunk_ref(a, buf, sz, L);
            else
                oracle_acc_add_chunk_spec(a, buf, sz, L);
        }
        free(buf);
    }
    oracle_reader_free(rd);
    int64_t m = oracle_acc_finish(a, out);
    oracle_acc_free(a);
    return m;
}

/* ------------------------------------------------------------------------- */
/* window checksums: a parity property for inputs too large to recount       */
/* ------------------------------------------------------------------------- */
/*
 * For a full-size run the output is a multiset {key: count}. Two 64-bit hash
 * functions h1, h2 (splitmix/murmur finalizers with different seeds) give
 *     sum over every valid window w of h(key(w))   (mod 2^64)
 *  == sum over every output record r of count(r) * h(key(r))   (mod 2^64)
 * for a correct output; a count moved between keys, a wrong key, a lost or an
 * extra window changes both sums unless the difference happens to cancel in
 * both hashes (~2^-128 for errors independent of the hashes). Together with
 * strictly ascending keys, the count sum and the key-0 rule below this pins the
 * output at any size in seconds on the host's cores.
 *
 * Windows follow the spec form (o_spec_key, SURVEY Appendix A, which restates
 * GPUHandler.cu:129-233): each read of well-formed 4-line FASTQ at its own
 * length; a window holding a byte outside ACGT is invalid (the zeroed hole
 * record of extractKMers: it only makes key 0^W present, count 0).
 */

static uint64_t o_ck_hash(const uint64_t* key, int W, uint64_t seed) {
    uint64_t h = seed;
    for (int j = 0; j < W; j++) h = o_mix64(h ^ key[j]) + 0x9e3779b97f4a7c15ull * (uint64_t)(j + 1);
    return o_mix64(h ^ (uint64_t)W);
}

#define O_CK_SEED1 0x243f6a8885a308d3ull
#define O_CK_SEED2 0x13198a2e03707344ull

typedef struct o_ck_job {
    const unsigned char* p;
    int64_t n, lo, hi; /* records starting in [lo, hi) */
    int64_t k;
    uint64_t s1, s2, windows, valid, hole, reads;
} o_ck_job;

/* the first record start at or after `from`: a line starting with '@' whose
 * next-but-one line starts with '+' (a quality line starting with '@' is
 * followed by a header and a sequence, never by a '+' two lines on) */
static int64_t o_ck_record_start(const unsigned char* p, int64_t n, int64_t from) {
    int64_t i = from;
    if (i > 0 && i < n && p[i - 1] != '\n') {
        const unsigned char* nl = (const unsigned char*)memchr(p + i, '\n', (size_t)(n - i));
        if (!nl) return n;
        i = (nl - p) + 1;
    }
    while (i < n) {
        if (p[i] == '@') {
            const unsigned char* a = (const unsigned char*)memchr(p + i, '\n', (size_t)(n - i));
            const unsigned char* b = a ? (const unsigned char*)memchr(a + 1, '\n', (size_t)(n - (a + 1 - p))) : NULL;
            if (b && b + 1 < p + n && b[1] == '+') return i;
            if (!a) return n;
        }
        const unsigned char* nl = (const unsigned char*)memchr(p + i, '\n', (size_t)(n - i));
        if (!nl) return n;
        i = (nl - p) + 1;
    }
    return n;
}

static void* o_ck_worker(void* arg) {
    o_ck_job* j = (o_ck_job*)arg;
    const unsigned char* p = j->p;
    int64_t k = j->k, i = j->lo;
    int W = o_words(k);
    uint64_t mask_last = o_masks_last_word(k) ? (~0ull << (64 - 2 * (k % 32))) : ~0ull;
    uint64_t* w = NULL;
    int64_t wcap = 0;
    uint64_t key[O_MAXW];
    while (i < j->hi) {
        const unsigned char* a = (const unsigned char*)memchr(p + i, '\n', (size_t)(j->n - i));
        if (!a) break;
        const unsigned char* s = a + 1;
        const unsigned char* e = (const unsigned char*)memchr(s, '\n', (size_t)(j->n - (s - p)));
        if (!e) break;
        int64_t L = e - s;
        /* skip the '+' line and the quality line */
        const unsigned char* q = (const unsigned char*)memchr(e + 1, '\n', (size_t)(j->n - (e + 1 - p)));
        const unsigned char* r = q ? (const unsigned char*)memchr(q + 1, '\n', (size_t)(j->n - (q + 1 - p))) : NULL;
        i = r ? (r - p) + 1 : j->n;
        j->reads++;
        if (L < k) continue;
        if (L + 32 * W + 1 > wcap) {
            wcap = L + 32 * W + 64;
            free(w);
            w = (uint64_t*)calloc((size_t)wcap, 8);
        }
        /* w[x] = the 32 bases from x (MSB first), 0 past the read end */
        for (int64_t x = L; x < L + 32 * W + 1; x++) w[x] = 0;
        for (int64_t x = L - 1; x >= 0; x--) w[x] = ((uint64_t)o_code(s[x]) << 62) | (w[x + 1] >> 2);
        int64_t last_bad = -1;
        for (int64_t x = 0; x < k - 1; x++)
            if (o_bad(s[x])) last_bad = x;
        for (int64_t pp = 0; pp + k <= L; pp++) {
            if (o_bad(s[pp + k - 1])) last_bad = pp + k - 1;
            j->windows++;
            if (last_bad >= pp) {
                j->hole = 1;
                continue;
            }
            j->valid++;
            for (int t = 0; t < W; t++) key[t] = w[pp + 32 * t];
            key[W - 1] &= mask_last;
            j->s1 += o_ck_hash(key, W, O_CK_SEED1);
            j->s2 += o_ck_hash(key, W, O_CK_SEED2);
        }
    }
    free(w);
    return NULL;
}

/* out[0..5] = sum h1, sum h2, windows, valid windows, any invalid window (0/1),
 * reads. Returns 0, or -1 on bad arguments. */
int oracle_window_checksum(const char* fastq, int64_t n_bytes, int64_t k, int threads, uint64_t* out) {
    if (k < 1 || k > 32 * O_MAXW || threads < 1) return -1;
    const unsigned char* p = (const unsigned char*)fastq;
    o_ck_job* jobs = (o_ck_job*)calloc((size_t)threads, sizeof(o_ck_job));
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    int64_t prev = o_ck_record_start(p, n_bytes, 0);
    for (int t = 0; t < threads; t++) {
        int64_t hi = t + 1 == threads ? n_bytes : o_ck_record_start(p, n_bytes, n_bytes / threads * (t + 1));
        if (hi < prev) hi = prev;
        jobs[t].p = p;
        jobs[t].n = n_bytes;
        jobs[t].lo = prev;
        jobs[t].hi = hi;
        jobs[t].k = k;
        prev = hi;
        pthread_create(&th[t], NULL, o_ck_worker, &jobs[t]);
    }
    memset(out, 0, 6 * sizeof(uint64_t));
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        out[0] += jobs[t].s1;
        out[1] += jobs[t].s2;
        out[2] += jobs[t].windows;
        out[3] += jobs[t].valid;
        out[4] |= jobs[t].hole;
        out[5] += jobs[t].reads;
    }
    free(th);
    free(jobs);
    return 0;
}

typedef struct o_rck_job {
    const unsigned char* recs;
    int64_t lo, hi;
    int W;
    uint64_t s1, s2, cnt, unordered;
} o_rck_job;

static void* o_rck_worker(void* arg) {
    o_rck_job* j = (o_rck_job*)arg;
    int W = j->W, rs = 8 * W + 4;
    uint64_t key[O_MAXW], prev[O_MAXW];
    for (int64_t i = j->lo; i < j->hi; i++) {
        const unsigned char* r = j->recs + (size_t)i * rs;
        memcpy(key, r, (size_t)W * 8);
        uint32_t c;
        memcpy(&c, r + 8 * W, 4);
        if (i > 0) {
            memcpy(prev, r - rs, (size_t)W * 8);
            if (o_cmp_words(prev, key, W) >= 0) j->unordered++;
        }
        j->s1 += (uint64_t)c * o_ck_hash(key, W, O_CK_SEED1);
        j->s2 += (uint64_t)c * o_ck_hash(key, W, O_CK_SEED2);
        j->cnt += c;
    }
    return NULL;
}

/* Over n SortedKMerFile records (W LE u64 words + LE u32 count):
 * out[0..3] = sum count*h1, sum count*h2, sum count, adjacent pairs not
 * strictly ascending. */
int oracle_records_checksum(const unsigned char* recs, int64_t n, int64_t k, int threads, uint64_t* out) {
    if (k < 1 || k > 32 * O_MAXW || threads < 1 || n < 0) return -1;
    o_rck_job* jobs = (o_rck_job*)calloc((size_t)threads, sizeof(o_rck_job));
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 0; t < threads; t++) {
        jobs[t].recs = recs;
        jobs[t].lo = n / threads * t;
        jobs[t].hi = t + 1 == threads ? n : n / threads * (t + 1);
        jobs[t].W = o_words(k);
        pthread_create(&th[t], NULL, o_rck_worker, &jobs[t]);
    }
    memset(out, 0, 4 * sizeof(uint64_t));
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        out[0] += jobs[t].s1;
        out[1] += jobs[t].s2;
        out[2] += jobs[t].cnt;
        out[3] += jobs[t].unordered;
    }
    free(th);
    free(jobs);
    return 0;
}
