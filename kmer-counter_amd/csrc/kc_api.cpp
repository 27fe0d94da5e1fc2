// kc_api.cpp — the C ABI of include/kc.h: device context, buffers, the count
// pipeline (FASTQ index -> count_kmers -> spill runs) and the finish pipeline
// (compact -> radix sort -> pack -> merge with spill runs).
//
// Replaces PrepareGPU / processKMers / FreeGPU (GPUHandler.cu:397-519) and the
// host aggregation of KMerCounter (KMerCounter.cpp:51-106).
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <sched.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kc.h"
#include "kc_device.h"
#include "kc_io.h"
#include "kc_stage.h"

using namespace kc;

namespace {

std::atomic<uint64_t> g_ctx_seq(0);

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct HostRun {
    std::vector<uint8_t> mem;  // used when no temp dir
    std::string path;          // used with a temp dir
    uint64_t records = 0;
};

}  // namespace

struct kc_ctx {
    kc_config cfg;
    std::string temp_dir;
    int W = 1, rs = 12;
    int64_t k = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev2 = nullptr;  // a third mark: two phases timed by one synchronisation
    hipEvent_t evf[2] = {nullptr, nullptr};  // kc_finish's own marks (the passes inside it use ev0..ev2)
    double finish_group_ms = 0;              // the finish's grouping passes (histograms + scatters)
    uint64_t id = 0;

    // table + spill (the gpu_memory_limit working set)
    uint64_t* table = nullptr;
    uint64_t cap = 0;
    size_t table_bytes = 0;
    bool table_dirty = true;  // a slot may be non-zero (cleared by kc_reset)
    uint64_t* spill = nullptr;
    uint64_t spill_cap = 0;
    uint64_t* stats = nullptr;      // device ST_N
    uint64_t* stats_h = nullptr;    // pinned host mirror

    // partition engine (default): key buffers for one batch, records
    bool part = true;
    bool skm = false;              // KC_FLAG_ENGINE_SKM: super-k-mer records instead of keys
    bool skm_used = false;         // a batch went through the skm engine since the last reset
    bool skm_force = false;        // KC_FLAG_ENGINE_SKM: no cardinality sample
    bool skm_checked = false;      // the skm cardinality sample has run since the last reset
    bool skm_big_off = false;      // a large skm batch overflowed the spill or record buffer: safe batches only
    uint32_t engines_used = 0;     // kc_stats.engines_used
    bool skm_hc = false;           // high cardinality seen: the key-prefix engine counts
    bool hc_hint = false;          // most keys were distinct (the skm sample or the last key-prefix batch):
                                   // P5 splits buckets by their key count up front
    uint64_t* pool_cursor = nullptr;  // device u64: skm pool allocator
    uint64_t key_cap = 0;          // keys per batch
    uint64_t* keys_a = nullptr;    // W x key_cap
    uint8_t* digs = nullptr;       // digs_bytes: P3 digit (word0 >> 56) of keys_a[i], written by P2; the skm
                                   // engine keeps two digit bytes per record (both grouping passes)
    uint64_t digs_bytes = 0;
    uint64_t* keys_b = nullptr;
    DevBuf part_hist, part_base, part_tmp, part_starts, part_sort_hist;
    DevBuf part_ghist;  // key-range passes: P1 histogram by 16 key groups (+ the group totals)
    DevBuf part_base2;  // key-range passes: the second pass of a walk's run starts
    DevBuf part_dedup;  // skm P5a: per-bucket list starts (u64) and lengths (u32), list cursor
    DevBuf p3b_buf, sub_starts;  // key-prefix engine, high cardinality: P3b tile positions, sub-bucket starts
    DevBuf run_flags;            //   P5s: runs left to the LDS hash path
    DevBuf part_codes, part_inval;  // kernel E output: the batch's reads, 2-bit encoded
    DevBuf part_rlen;               // KC_FLAG_VARLEN: each read's own length (u16)
    const uint16_t* var_rlen = nullptr;  // set while a variable-length block is counted
    // P5 segment descriptors (see finish_part_sorted) and their sort scratch
    DevBuf desc_key, desc_start, desc_len, desc_k2, desc_v, desc_v2, desc_lens, desc_offs, desc_fb;
    uint64_t* rec_keys = nullptr;  // W x rec_cap
    uint8_t* rec_dig = nullptr;    // rec_cap: word 0 bits 48..55 of each record the skm P5 wrote (the
                                   // finish's first grouping digit, read as 1 B instead of word 0)
    uint32_t* rec_cnts = nullptr;
    uint64_t rec_cap = 0;
    uint64_t* rec_cursor = nullptr;  // device u64
    uint64_t rec_n = 0;              // host copy after each batch
    uint64_t batches = 0;
    int n_cu = 256;
    double part_ms[5] = {0, 0, 0, 0, 0};  // E+P1, P2, P3 scatter, P3 hist + P4, P5
    double presplit_ms = 0;                 // P3b (also in part_ms[2])
    uint64_t presplit_batches = 0, sorted_run_batches = 0, key_passes = 0;
    double dedup_ms = 0;                  // skm P5a
    uint64_t dedup_records = 0;
    uint64_t part_keys = 0;               // keys partitioned since the last reset
    uint64_t p5_launches = 0;

    // scratch (grown on demand)
    DevBuf in_stage;        // host-pointer inputs
    DevBuf fq_counts, fq_base, fq_tmp, seq_off, seq_end;
    DevBuf fq_phase;  // one-pass index: each chunk's guessed line phase
    DevBuf spill_keys2, rle_flags, rle_pos, rle_head, rle_tmp, run_keys, run_cnts, run_packed;
    DevBuf fin_keys[2], fin_cnts[2], fin_hist, fin_packed, fin_misc;
    DevBuf merge_tmp;  // packed run merge: the other ping-pong buffer

    // host staging (kc_stage.h), created on the first host-pointer input or output
    kc::Pool* pool = nullptr;
    kc::PinnedRing* ring = nullptr;
    std::vector<char*> file_bufs;  // pinned blocks of kc_count_file's reader (kept: pinning is slow)
    size_t file_buf_bytes = 0;
    hipStream_t copy_stream = nullptr;  // kc_count_file: block i+1 uploads while block i is decoded
    hipEvent_t file_ev[2] = {nullptr, nullptr};
    hipEvent_t stage_free[2] = {nullptr, nullptr};  // kc_count_chunk: the encode of the staged chunk is done
    DevBuf file_stage[2];
    int chunk_slot = 0;
    // kc_count_chunk accumulation: whole reads of consecutive chunks copied
    // into one of two pinned buffers, uploaded and encoded when it fills (or
    // before anything else counts, finishes or checkpoints)
    char* acc_buf[2] = {nullptr, nullptr};
    hipEvent_t acc_ev[2] = {nullptr, nullptr};
    bool acc_busy[2] = {false, false};
    size_t acc_n = 0;
    int acc_i = 0;
    int64_t acc_L = 0;
    double acc_t[4] = {0, 0, 0, 0};  // KC_TRACE: host copy, buffer wait, flush, calls (s)

    // Pending batch: reads already indexed and 2-bit encoded into part_codes /
    // part_inval (/ part_rlen) by kc_count_* calls, counted together at the
    // next flush (when the next block does not fit, its read length differs,
    // or at kc_finish). Many small calls thus count as one batch.
    int64_t pend_L = 0;
    bool pend_var = false;
    uint64_t pend_reads = 0;
    // the pending rows hold one-pass-indexed blocks (rows per chunk, empty rows
    // of length 0): every pending row has its length in part_rlen, the skm
    // front end reads them, and key 0's presence is recomputed at the flush
    // from ST_VHOLE as for variable-length reads
    bool pend_sparse = false;
    uint64_t flush_present0 = 0;  // key 0's presence before the flush of padded / one-pass rows
    uint64_t flushes = 0;
    uint64_t dev_total = 0;  // device memory (bytes)
    // kc_checkpoint / kc_rollback: the pending state and the counters a
    // rolled-back block may have changed
    bool ckpt = false;
    uint64_t ckpt_reads = 0, ckpt_flushes = 0, ckpt_st_reads = 0, ckpt_st_windows = 0;
    uint64_t ckpt_stats[ST_N];

    // Sorted runs cut from the records when they outgrow half the working set
    // (cut_run): kept in HBM outside the counting working set (host memory
    // only when HBM is short, as c->runs), merged on the device by kc_finish
    std::vector<DevBuf> dev_runs;
    std::vector<uint64_t> dev_run_n;
    std::vector<DevBuf> run_pool;  // run buffers of earlier counts, reused (allocations are kept like all others)
    uint64_t runs_cut = 0;
    uint64_t batches_cut = 0;  // batches of the records already cut into runs

    // results
    bool finished = false;
    uint64_t n_records = 0;  // table run
    uint64_t spilled_flushed = 0;
    std::vector<HostRun> runs;

    kc_stats st;
    std::string err;
};

static kc_status cut_run(kc_ctx* c);
static kc_status recompute_presence(kc_ctx* c);
static kc_status keep_finished_run(kc_ctx* c, uint64_t n);
static kc_status cut_run_if_full(kc_ctx* c);
static kc_status merge_runs_list(kc_ctx* c, const std::vector<std::pair<const void*, uint64_t>>& runs);
static kc_status merge_runs_packed(kc_ctx* c, const std::vector<std::pair<const void*, uint64_t>>& runs);
static void release_dev_runs(kc_ctx* c, bool free_pool);

static kc_status fail(kc_ctx* c, kc_status s, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return s;
}

// The host-side counters one batch adds to (kc_stats timings and launch
// counts, engine flags): snapshot before a batch that may be undone.
struct HostCounters {
    uint64_t insert_launches;
    double insert_ms;
    double part_ms[5];
    double dedup_ms;
    uint64_t p5_launches, part_keys;
    bool skm_used, skm_checked;
    uint32_t engines_used;
};

static HostCounters host_counters(const kc_ctx* c) {
    HostCounters h;
    h.insert_launches = c->st.insert_launches;
    h.insert_ms = c->st.insert_ms;
    memcpy(h.part_ms, c->part_ms, sizeof(h.part_ms));
    h.dedup_ms = c->dedup_ms;
    h.p5_launches = c->p5_launches;
    h.part_keys = c->part_keys;
    h.skm_used = c->skm_used;
    h.skm_checked = c->skm_checked;
    h.engines_used = c->engines_used;
    return h;
}

static void restore_host_counters(kc_ctx* c, const HostCounters& h) {
    c->st.insert_launches = h.insert_launches;
    c->st.insert_ms = h.insert_ms;
    memcpy(c->part_ms, h.part_ms, sizeof(h.part_ms));
    c->dedup_ms = h.dedup_ms;
    c->p5_launches = h.p5_launches;
    c->part_keys = h.part_keys;
    c->skm_used = h.skm_used;
    c->skm_checked = h.skm_checked;
    c->engines_used = h.engines_used;
}

#define HIPCHK(ctx, expr)                                                                                    \
    do {                                                                                                     \
        hipError_t e_ = (expr);                                                                              \
        if (e_ != hipSuccess)                                                                                \
            return fail((ctx), e_ == hipErrorOutOfMemory ? KC_ERR_NOMEM : KC_ERR_HIP, "%s: %s (%s:%d)", #expr, \
                        hipGetErrorString(e_), __FILE__, __LINE__);                                          \
    } while (0)

static kc_status ensure(kc_ctx* c, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return KC_OK;
    if (b.p) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(b.p));
        b.p = nullptr;
        b.bytes = 0;
    }
    size_t want = bytes < 256 ? 256 : bytes;
    HIPCHK(c, hipMalloc(&b.p, want));
    b.bytes = want;
    return KC_OK;
}

// As ensure, but a pooled run buffer that is big enough (best fit) is swapped
// in before anything is allocated: finished runs, merge outputs and fin_packed
// trade the same few large buffers instead of reallocating tens of GB per pass.
static kc_status ensure_pooled(kc_ctx* c, DevBuf& b, size_t bytes) {
    if (b.p && b.bytes >= bytes) return KC_OK;
    int best = -1;
    for (size_t i = 0; i < c->run_pool.size(); i++)
        if (c->run_pool[i].bytes >= bytes && (best < 0 || c->run_pool[i].bytes < c->run_pool[(size_t)best].bytes))
            best = (int)i;
    if (best >= 0) {
        DevBuf t = c->run_pool[(size_t)best];
        c->run_pool.erase(c->run_pool.begin() + best);
        if (b.p) c->run_pool.push_back(b);
        b = t;
        return KC_OK;
    }
    return ensure(c, b, bytes);
}

static void release(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

static kc_status sync_stats(kc_ctx* c) {
    HIPCHK(c, hipMemcpyAsync(c->stats_h, c->stats, ST_N * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return KC_OK;
}

static uint32_t probe_limit(const kc_ctx* c) {
    // a nearly full table: give up early and spill instead of walking long runs
    uint64_t used = c->stats_h[ST_CLAIMED];
    if (used * 10 >= c->cap * 9) return 8;
    return c->W == 1 ? 128 : 64;
}

// ---------------------------------------------------------------------------
// sorting helpers (device)
// ---------------------------------------------------------------------------

// Sorts n SoA records (keys at `stride`) in place-or-swap; returns which buffer
// holds the result (0 = a, 1 = b).
static kc_status sort_records(kc_ctx* c, uint64_t* ka, uint64_t* kb, uint32_t* va, uint32_t* vb, uint64_t stride,
                              uint64_t n, int* which, int words = 0) {
    *which = 0;
    if (n <= 1) return KC_OK;
    const int W = words ? words : c->W;
    kc_status s = ensure(c, c->fin_misc, 2 * W * 8);
    if (s) return s;
    std::vector<uint64_t> init(2 * W);
    for (int j = 0; j < W; j++) {
        init[j] = 0;
        init[W + j] = ~0ull;
    }
    HIPCHK(c, hipMemcpyAsync(c->fin_misc.p, init.data(), 2 * W * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_key_bits(W, ka, stride, n, (uint64_t*)c->fin_misc.p, c->stream));
    std::vector<uint64_t> bits(2 * W);
    HIPCHK(c, hipMemcpyAsync(bits.data(), c->fin_misc.p, 2 * W * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int grid = sort_grid(n);
    s = ensure(c, c->fin_hist, (size_t)sort_hist_elems(grid) * 8);
    if (s) return s;
    uint64_t* kin = ka;
    uint64_t* kout = kb;
    uint32_t* vin = va;
    uint32_t* vout = vb;
    int cur = 0;
    for (int word = W - 1; word >= 0; word--) {
        uint64_t vary = bits[word] ^ bits[W + word];
        for (int shift = 0; shift < 64; shift += 8) {
            if (((vary >> shift) & 255u) == 0) continue;
            HIPCHK(c, launch_sort_pass(W, kin, kout, vin, vout, stride, n, word, shift, (uint64_t*)c->fin_hist.p,
                                       grid, false, c->stream));
            std::swap(kin, kout);
            std::swap(vin, vout);
            cur ^= 1;
        }
    }
    *which = cur;
    return KC_OK;
}

// ---------------------------------------------------------------------------
// spill runs: sort the spill buffer, run-length reduce, pack, move to host
// ---------------------------------------------------------------------------

// A sorted packed run of n records (device memory, rewritten later) kept as a
// device run when HBM has room for it plus a margin; false: the caller keeps
// it on the host.
static bool keep_run_on_device(kc_ctx* c, const void* packed, uint64_t n) {
    const size_t bytes = (size_t)n * c->rs;
    size_t mfree = 0, mtotal = 0;
    DevBuf run;
    if (hipMemGetInfo(&mfree, &mtotal) != hipSuccess || mfree < bytes + ((size_t)4 << 30) ||
        hipMalloc(&run.p, bytes ? bytes : 16) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    run.bytes = bytes;
    if (hipMemcpyAsync(run.p, packed, bytes, hipMemcpyDeviceToDevice, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        (void)hipFree(run.p);
        (void)hipGetLastError();
        return false;
    }
    c->dev_runs.push_back(run);
    c->dev_run_n.push_back(n);
    c->runs_cut++;
    return true;
}

// Sorts n spilled keys (SoA at `stride` in `keys`, `scratch` of the same
// shape), run-length reduces them and stores the run (host memory or a temp
// file).
static kc_status flush_keys(kc_ctx* c, uint64_t* keys, uint64_t stride, uint64_t n, uint64_t* scratch) {
    kc_status s;
    const int W = c->W;
    int which = 0;
    if ((s = sort_records(c, keys, scratch, nullptr, nullptr, stride, n, &which))) return s;
    uint64_t* sorted = which ? scratch : keys;
    if ((s = ensure(c, c->rle_flags, n * 4)) || (s = ensure(c, c->rle_pos, n * 4)) ||
        (s = ensure(c, c->rle_head, n * 4)) || (s = ensure(c, c->rle_tmp, scan_tmp_elems(n) * 4)) ||
        (s = ensure(c, c->run_keys, (size_t)W * n * 8)) || (s = ensure(c, c->run_cnts, n * 4)))
        return s;
    HIPCHK(c, launch_rle_heads(W, sorted, stride, n, (uint32_t*)c->rle_flags.p, c->stream));
    HIPCHK(c, launch_scan_u32((uint32_t*)c->rle_flags.p, (uint32_t*)c->rle_pos.p, n, (uint32_t*)c->rle_tmp.p,
                              c->stream));
    uint32_t last[2];
    HIPCHK(c, hipMemcpyAsync(&last[0], (uint32_t*)c->rle_pos.p + (n - 1), 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&last[1], (uint32_t*)c->rle_flags.p + (n - 1), 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    uint64_t m = (uint64_t)last[0] + last[1];
    HIPCHK(c, launch_rle_scatter(W, sorted, stride, n, (uint32_t*)c->rle_flags.p, (uint32_t*)c->rle_pos.p,
                                 (uint64_t*)c->run_keys.p, n, (uint32_t*)c->rle_head.p, c->stream));
    HIPCHK(c, launch_rle_counts((uint32_t*)c->rle_head.p, m, n, (uint32_t*)c->run_cnts.p, c->stream));
    size_t bytes = (size_t)m * c->rs;
    if ((s = ensure(c, c->run_packed, bytes))) return s;
    HIPCHK(c, launch_pack(W, (uint64_t*)c->run_keys.p, n, (uint32_t*)c->run_cnts.p, m, c->run_packed.p, c->stream));
    c->spilled_flushed += n;
    // the run stays in HBM (merged on the device by kc_finish) unless HBM is
    // short: then host memory, or a file in tempFileLocation
    if (keep_run_on_device(c, c->run_packed.p, m)) return KC_OK;
    HostRun run;
    run.records = m;
    run.mem.resize(bytes);
    HIPCHK(c, hipMemcpyAsync(run.mem.data(), c->run_packed.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (!c->temp_dir.empty()) {
        char name[128];
        snprintf(name, sizeof(name), "/kc.%d.%llu.%zu", (int)getpid(), (unsigned long long)c->id, c->runs.size());
        run.path = c->temp_dir + name;
        FILE* f = fopen(run.path.c_str(), "wb");
        if (!f) return fail(c, KC_ERR_IO, "cannot create spill run %s: %s", run.path.c_str(), strerror(errno));
        size_t w = fwrite(run.mem.data(), 1, bytes, f);
        const int we = errno;
        const int ce = fclose(f) != 0 ? errno : 0;
        if (w != bytes || ce)
            return fail(c, KC_ERR_IO, "short write to spill run %s (%zu of %llu bytes): %s", run.path.c_str(), w,
                        (unsigned long long)bytes, strerror(w != bytes ? we : ce));
        std::vector<uint8_t>().swap(run.mem);
    }
    c->runs.push_back(std::move(run));
    c->st.spill_runs = c->runs.size();
    return KC_OK;
}

// Flushes the spill buffer of the global table into a sorted run.
static kc_status flush_spill(kc_ctx* c) {
    kc_status s = sync_stats(c);
    if (s) return s;
    uint64_t n = c->stats_h[ST_SPILL_FILL];
    if (n == 0) return KC_OK;
    if (n > c->spill_cap) return fail(c, KC_ERR_INTERNAL, "spill buffer overflow (%llu > %llu)",
                                      (unsigned long long)n, (unsigned long long)c->spill_cap);
    if ((s = ensure(c, c->spill_keys2, (size_t)c->W * c->spill_cap * 8))) return s;
    if ((s = flush_keys(c, c->spill, c->spill_cap, n, (uint64_t*)c->spill_keys2.p))) return s;
    HIPCHK(c, hipMemsetAsync(c->stats + ST_SPILL_FILL, 0, 8, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->stats_h[ST_SPILL_FILL] = 0;
    return KC_OK;
}

// ---------------------------------------------------------------------------
// counting
// ---------------------------------------------------------------------------

static kc_status check_line(kc_ctx* c, int64_t L) {
    if (L < c->k) return fail(c, KC_ERR_ARG, "read length %lld is shorter than k=%lld", (long long)L, (long long)c->k);
    if (L > 32767) return fail(c, KC_ERR_ARG, "read length %lld exceeds 32767 (the reference's u16 2L header)",
                               (long long)L);
    return KC_OK;
}

// Engine "table": every k-mer is inserted into the global HBM table with
// atomics. Counts n_reads reads (stride mode when seq_off == nullptr).
static kc_status count_reads_table(kc_ctx* c, const uint8_t* base, const uint64_t* seq_off, uint64_t n_reads,
                                   int64_t L) {
    if (c->finished) return fail(c, KC_ERR_STATE, "kc_finish was called; kc_reset first");
    const uint64_t nw = (uint64_t)(L - c->k + 1);
    const uint64_t max_reads = c->spill_cap / nw;
    if (max_reads == 0) return fail(c, KC_ERR_ARG, "gpu_memory_limit too small for one read's windows");
    uint64_t done = 0;
    kc_status s;
    float ms = 0.f;
    while (done < n_reads) {
        uint64_t free_slots = c->spill_cap - c->stats_h[ST_SPILL_FILL];
        uint64_t nr = n_reads - done;
        if (nr > max_reads) nr = max_reads;
        if (nr * nw > free_slots) {
            if ((s = flush_spill(c))) return s;
        }
        CountLaunch a;
        a.base = base;
        a.seq_off = seq_off;
        a.read0 = done;
        a.n_reads = nr;
        a.L = (int)L;
        a.k = (int)c->k;
        a.table = c->table;
        a.cap = c->cap;
        a.spill = c->spill;
        a.spill_cap = c->spill_cap;
        a.stats = c->stats;
        a.probe_limit = probe_limit(c);
        HIPCHK(c, hipEventRecord(c->ev0, c->stream));
        HIPCHK(c, launch_count_kmers(a, 256 * 16, c->stream));
        HIPCHK(c, hipEventRecord(c->ev1, c->stream));
        if ((s = sync_stats(c))) return s;
        float t = 0.f;
        HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
        ms += t;
        c->st.insert_launches++;
        if (c->stats_h[ST_ERR] & ERR_SPILL_OVERFLOW) return fail(c, KC_ERR_INTERNAL, "spill buffer overflow");
        done += nr;
    }
    c->st.insert_ms += ms;
    c->st.last_count_ms = ms;
    c->engines_used |= 4u;
    c->st.valid_kmers = c->stats_h[ST_VALID];
    c->st.spilled_kmers = c->spilled_flushed + c->stats_h[ST_SPILL_FILL];
    return KC_OK;
}

static kc_status grow_records(kc_ctx* c, uint64_t need) {
    if (need <= c->rec_cap) return KC_OK;
    uint64_t ncap = c->rec_cap ? c->rec_cap : 1024;
    while (ncap < need) ncap = ncap + ncap / 2 + 1024;
    const int W = c->W;
    uint64_t* nk = nullptr;
    uint32_t* nc = nullptr;
    uint8_t* nd = nullptr;
    HIPCHK(c, hipMalloc((void**)&nk, (size_t)W * ncap * 8));
    HIPCHK(c, hipMalloc((void**)&nc, (size_t)ncap * 4));
    HIPCHK(c, hipMalloc((void**)&nd, (size_t)ncap + 16));
    if (c->rec_n) {
        for (int j = 0; j < W; j++)
            HIPCHK(c, hipMemcpyAsync(nk + (size_t)j * ncap, c->rec_keys + (size_t)j * c->rec_cap, c->rec_n * 8,
                                     hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(nc, c->rec_cnts, c->rec_n * 4, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(nd, c->rec_dig, c->rec_n, hipMemcpyDeviceToDevice, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->rec_keys) HIPCHK(c, hipFree(c->rec_keys));
    if (c->rec_cnts) HIPCHK(c, hipFree(c->rec_cnts));
    if (c->rec_dig) HIPCHK(c, hipFree(c->rec_dig));
    c->rec_keys = nk;
    c->rec_cnts = nc;
    c->rec_dig = nd;
    c->rec_cap = ncap;
    return KC_OK;
}

static const int kBucketBits = 16;
static const size_t kMaxLds = 160 * 1024;  // LDS of one CU (gfx950): the P2 workgroup's ceiling
static const uint64_t kDescCap = 1u << 20;  // P5 segment descriptors kept for the sorted finish
// skm engine cardinality sample: buckets counted first, the smallest batch
// (keys) sampled, and the distinct-key share above which the key-prefix engine
// counts instead
static const uint32_t kSkmSample = 256;
static const uint64_t kSkmSampleMinKeys = 1ull << 24;
static const double kSkmDistinctMax = 0.35;

// P5s direct (high cardinality, empty record state): sort_runs_k writes the
// batch's records straight into fin_packed as a finished sorted run (record
// 0: key 0 when present), each run of sub-buckets at its first key's position;
// runs that held equal keys leave gaps that a segment copy closes. With
// key-range passes (count_reads_part) every pass appends its key range at
// record pk_at (the records of the earlier passes); `last` keeps fin_packed as
// the finished run (direct_keep) and the record state stays empty. *done =
// false when runs were handed to the hash path: nothing of this batch was
// kept and the caller counts it into records as usual. `total` sizes
// fin_packed on the first pass (keys of all passes).
static kc_status direct_keep(kc_ctx* c, uint64_t nrec);
static kc_status p5s_direct(kc_ctx* c, const uint64_t* keys, uint64_t kstride, const uint64_t* sub_starts, uint32_t nb,
                            uint64_t n,
                            uint8_t* rf, size_t fl, bool* done, uint64_t* records, float* ms, uint64_t pk_at = 0,
                            uint64_t total = 0, bool last = true) {
    kc_status s;
    *done = false;
    const int W = c->W;
    const size_t rs = (size_t)c->rs;
    uint8_t* bf = rf + ((size_t)nb << 8);
    uint32_t* nflag = (uint32_t*)(bf + nb);
    // (inside a flush of padded / one-pass rows: key 0's presence from the reads)
    if ((s = c->var_rlen ? recompute_presence(c) : sync_stats(c))) return s;
    const bool key0 = c->stats_h[ST_KEY0_PRESENT] != 0;
    const uint64_t off0 = key0 ? 1 : 0;
    if (pk_at == 0 && (s = ensure_pooled(c, c->fin_packed, (off0 + (total > n ? total : n)) * rs + 16))) return s;
    if (c->fin_packed.bytes < (off0 + pk_at + n) * rs) return fail(c, KC_ERR_INTERNAL, "key-range pass overflows its run");
    HIPCHK(c, hipMemsetAsync(rf, 0, fl, c->stream));
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, launch_sort_runs(W, keys, kstride, sub_starts, nb, c->rec_keys, c->rec_cnts, c->rec_cap,
                               c->rec_cursor, c->stats, (uint64_t*)c->desc_key.p, (uint64_t*)c->desc_start.p,
                               (uint32_t*)c->desc_len.p, kDescCap, rf, bf, nflag, 2 * c->n_cu, c->stream,
                               c->fin_packed.p, off0 + pk_at));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    uint32_t nf = 0;
    uint64_t R = 0;
    HIPCHK(c, hipMemcpyAsync(&nf, nflag, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&R, c->rec_cursor, 8, hipMemcpyDeviceToHost, c->stream));
    if ((s = sync_stats(c))) return s;
    HIPCHK(c, hipEventElapsedTime(ms, c->ev0, c->ev1));
    *records = R;
    const uint64_t ndesc = c->stats_h[ST_DESC_FILL];
    auto clear_cursor = [&]() -> kc_status {
        // record cursor and descriptors start empty again
        HIPCHK(c, hipMemsetAsync(c->rec_cursor, 0, 8, c->stream));
        c->stats_h[ST_DESC_FILL] = 0;
        HIPCHK(c, hipMemcpyAsync(c->stats + ST_DESC_FILL, &c->stats_h[ST_DESC_FILL], 8, hipMemcpyHostToDevice,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return KC_OK;
    };
    if (nf || (R < n && ndesc > kDescCap)) return clear_cursor();  // undo: the caller counts into records
    if (R < n) {
        // equal keys in some runs: close the gaps (segments in key order) into
        // merge_tmp, then back to the pass's place
        if ((s = ensure(c, c->desc_k2, ndesc * 8)) || (s = ensure(c, c->desc_v, ndesc * 4)) ||
            (s = ensure(c, c->desc_v2, ndesc * 4)) || (s = ensure(c, c->desc_lens, ndesc * 8)) ||
            (s = ensure(c, c->desc_offs, ndesc * 8)) || (s = ensure(c, c->rle_tmp, scan_tmp_elems(ndesc) * 8)) ||
            (s = ensure_pooled(c, c->merge_tmp, R * rs + 16)))
            return s;
        HIPCHK(c, launch_iota_u32((uint32_t*)c->desc_v.p, ndesc, c->stream));
        int which = 0;
        if ((s = sort_records(c, (uint64_t*)c->desc_key.p, (uint64_t*)c->desc_k2.p, (uint32_t*)c->desc_v.p,
                              (uint32_t*)c->desc_v2.p, ndesc, ndesc, &which, 1)))
            return s;
        const uint32_t* order = (const uint32_t*)(which ? c->desc_v2.p : c->desc_v.p);
        HIPCHK(c, launch_desc_prep(order, (const uint32_t*)c->desc_len.p, ndesc, (uint64_t*)c->desc_lens.p,
                                   c->stream));
        HIPCHK(c, launch_scan_u64((const uint64_t*)c->desc_lens.p, (uint64_t*)c->desc_offs.p, ndesc,
                                  (uint64_t*)c->rle_tmp.p, c->stream));
        HIPCHK(c, launch_packed_seg_copy(W, c->fin_packed.p, c->merge_tmp.p, order, (const uint64_t*)c->desc_start.p,
                                         (const uint32_t*)c->desc_len.p, (const uint64_t*)c->desc_offs.p, ndesc, 0,
                                         4 * c->n_cu, c->stream));
        HIPCHK(c, hipMemcpyAsync((uint8_t*)c->fin_packed.p + (off0 + pk_at) * rs, c->merge_tmp.p, R * rs,
                                 hipMemcpyDeviceToDevice, c->stream));
    }
    if ((s = clear_cursor())) return s;
    *done = true;
    return last ? direct_keep(c, pk_at + R) : KC_OK;
}

// fin_packed, written by direct passes (nrec records after the key-0 slot),
// becomes a finished sorted run
static kc_status direct_keep(kc_ctx* c, uint64_t nrec) {
    kc_status s;
    if ((s = c->var_rlen ? recompute_presence(c) : sync_stats(c))) return s;
    const bool key0 = c->stats_h[ST_KEY0_PRESENT] != 0;
    std::vector<uint32_t> r0((size_t)c->rs / 4, 0u);
    if (key0) {
        r0.back() = (uint32_t)c->stats_h[ST_KEY0];
        HIPCHK(c, hipMemcpyAsync(c->fin_packed.p, r0.data(), c->rs, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->batches = 1;  // this batch: moved to batches_cut with the run
    return keep_finished_run(c, (key0 ? 1 : 0) + nrec);
}

// Key-range passes (high cardinality): when one batch cannot hold the keys of
// all reads, the reads are not cut into batches whose sorted runs must then be
// merged; the key space is cut instead. A P1 pass over all reads counts the
// live keys by their top byte (word0 >> 56); consecutive top bytes are
// grouped into passes of at most key_cap keys, balanced; each pass re-walks all
// reads and keeps only its key range (P1/P2 filter), and P5s direct writes it
// after the previous passes' records: the runs are disjoint key ranges in key
// order, so the finished run is their concatenation (no merge). Returns the
// pass bounds (empty: not applicable, count by read batches).
static kc_status plan_key_passes(kc_ctx* c, CountLaunch l, int64_t L, std::vector<uint32_t>* kp, uint64_t* keys) {
    kp->clear();
    kc_status s;
    PartGeom pg = part_geometry((int)L, (int)c->k, l.n_reads);
    const uint64_t hn = 256 * pg.nseg;
    constexpr uint32_t NG = 16;  // key groups: word0 >> 60
    if ((s = ensure(c, c->part_ghist, (NG * hn + NG) * 8))) return s;
    uint64_t* gh = (uint64_t*)c->part_ghist.p;
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, launch_part_hist(l, pg, gh, 48, c->stream, 4));
    HIPCHK(c, launch_hist_group_totals(gh, pg.nseg, NG, gh + NG * hn, c->stream));
    std::vector<uint64_t> gt(NG);
    HIPCHK(c, hipMemcpyAsync(gt.data(), gh + NG * hn, NG * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float t = 0.f;
    HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
    c->part_ms[0] += t;
    uint64_t total = 0;
    for (uint64_t x : gt) total += x;
    *keys = total;
    if (total <= c->key_cap) return KC_OK;
    uint64_t np = (total + c->key_cap - 1) / c->key_cap;
    // (KC_KEY_PASSES_MIN: path selector for tests and measurements, same counts)
    if (const char* e = test_hook("KC_KEY_PASSES_MIN")) np = std::max<uint64_t>(np, strtoull(e, nullptr, 10));
    const uint64_t cap = std::min<uint64_t>(c->key_cap, (total + np - 1) / np * 5 / 4);
    const uint64_t target = (total + np - 1) / np;
    std::vector<uint32_t> bounds{0};
    uint64_t acc = 0;
    for (uint32_t g = 0; g < NG; g++) {
        const uint64_t x = gt[g];
        if (x > c->key_cap) return KC_OK;  // one group holds more than a batch: read batches
        // (a group above the balanced cap but within a batch gets a pass of its own)
        // close the pass before g when g would overflow it, or when stopping
        // here is closer to the balanced target than taking g
        if (acc > 0 && (acc + x > cap || (acc + x > target && acc + x - target > target - acc))) {
            bounds.push_back(g * (256 / NG));
            acc = 0;
        }
        acc += x;
    }
    bounds.push_back(256);
    if (bounds.size() - 1 > 16) return KC_OK;
    *kp = bounds;
    return KC_OK;
}

// Smallest batch (keys) that takes the P3b pre-split (high cardinality);
// KC_P3B_MIN: path selector for tests, same counts either way
static uint64_t p3b_min_of() {
    uint64_t m = 1ull << 22;
    if (const char* e = test_hook("KC_P3B_MIN")) m = strtoull(e, nullptr, 10);
    return m;
}

// Engine "partition": per batch of reads
//   P1 hist   : digit (word0 >> 48) & 255 per segment of reads
//   P2 scatter: keys to their digit's region (LDS counting sort per tile)
//   P3        : regional scatter on digit (word0 >> 56) -> grouped by bucket =
//               word0 >> 48, the key's first 8 bases: buckets are in key order
//   P4        : bucket ranges (binary search)
//   P5        : per-bucket LDS hash count -> (key, count) records
// pre0 >= 0: the reads are already encoded (fq_encode) in part_codes /
// part_inval from read index pre0 on; kernel E is skipped
static kc_status count_reads_part(kc_ctx* c, const uint8_t* base, const uint64_t* seq_off, uint64_t n_reads,
                                  int64_t L, int64_t pre0) {
    if (c->finished) return fail(c, KC_ERR_STATE, "kc_finish was called; kc_reset first");
    const int W = c->W;
    const uint64_t nw = (uint64_t)(L - c->k + 1);
    const uint64_t max_reads = c->key_cap / nw;
    if (max_reads == 0) return fail(c, KC_ERR_ARG, "gpu_memory_limit too small for one read's windows");
    kc_status s;
    uint64_t done = 0;
    float t = 0.f;
    const uint64_t G = (uint64_t)groups_per_read((int)L);
    auto launch_args = [&](uint64_t read0, uint64_t nr) {
        CountLaunch l;
        l.base = base;
        l.seq_off = seq_off;
        l.read0 = read0;
        l.n_reads = nr;
        l.L = (int)L;
        l.k = (int)c->k;
        l.table = c->table;
        l.cap = c->cap;
        l.spill = c->spill;
        l.spill_cap = c->spill_cap;
        l.stats = c->stats;
        l.probe_limit = probe_limit(c);
        const uint64_t g0 = pre0 < 0 ? 0 : ((uint64_t)pre0 + read0) * G;
        l.codes = (const uint32_t*)c->part_codes.p + g0;
        l.inval = (const uint16_t*)c->part_inval.p + g0;
        // rows of length 0 (one-pass empty rows) are skipped by P1 / P2
        l.rlen = (pre0 >= 0 && c->var_rlen) ? c->var_rlen + (uint64_t)pre0 + read0 : nullptr;
        return l;
    };
    // Key-range passes (plan_key_passes): high cardinality, all reads encoded,
    // more keys than one batch holds, and an empty record state (P5s direct)
    std::vector<uint32_t> kp;  // pass bounds on word0 >> 56
    size_t kpi = 0;            // current pass
    uint64_t kp_keys = 0;      // live keys of all passes
    uint64_t kp_out = 0;       // records the direct passes wrote so far
    bool kp_direct = false;    // every pass so far went direct
    // two passes per walk: P2 writes the second pass's keys (SoA, stride = its
    // key count, then its digit bytes) into fin_packed past the records the
    // first pass will write; that pass's P3 reads them from there
    size_t kp_u_pass = ~(size_t)0;  // the pass whose P2 output is at kp_u_keys
    uint64_t* kp_u_keys = nullptr;
    uint64_t kp_u_n = 0;
    // KC_P2_NO_DIGS (measurement): P2 writes no digit bytes (P3 reads word 0)
    const bool p2_no_digs = test_hook("KC_P2_NO_DIGS") != nullptr && !test_hook("KC_P3_SCATTER");
    // P2 writes each key as W consecutive words (one stream per digit run
    // instead of W) when P3 is the radix scatter, which reads them so
    // (KC_P2_SOA: the SoA layout, for comparison)
    const bool p2_aos =
        !p2_no_digs && !test_hook("KC_P2_SOA") && !test_hook("KC_P3_SCATTER") && p3_tile(W) == rp_tile(W, false);
    if (pre0 >= 0 && c->hc_hint && nw * n_reads > c->key_cap && c->rec_n == 0 && c->batches == 0 &&
        c->stats_h[ST_CLAIMED] == 0 && !c->skm_used && c->runs.empty() && !test_hook("KC_NO_KEY_PASSES") &&
        !test_hook("KC_NO_P3B") && !test_hook("KC_NO_SORT_RUNS") && !test_hook("KC_NO_P5S_DIRECT")) {
        if ((s = plan_key_passes(c, launch_args(0, n_reads), L, &kp, &kp_keys))) return s;
        kp_direct = !kp.empty();
        if (!kp.empty()) c->key_passes += kp.size() - 1;
        // the finished run's buffer (key 0 slot + every key), before the first
        // walk: it holds the second pass's P2 output until that pass's P3
        if (!kp.empty() && (s = ensure_pooled(c, c->fin_packed, (1 + kp_keys) * (size_t)c->rs + 16))) return s;
        if (getenv("KC_DEBUG") && !kp.empty())
            fprintf(stderr, "kc: %zu key-range passes over %llu keys\n", kp.size() - 1, (unsigned long long)kp_keys);
    }
    while (done < n_reads) {
        const bool kpass = !kp.empty();
        uint64_t nr = n_reads - done;
        if (nr > max_reads && !kpass) nr = max_reads;
        CountLaunch l = launch_args(done, nr);
        if (kpass) {
            l.flo = kp[kpi];
            l.fhi = kp[kpi + 1];
            l.no_stats = kpi > 0;
        }
        PartGeom pg = part_geometry((int)L, (int)c->k, nr);
        uint64_t hn = 256 * pg.nseg;
        if ((s = ensure(c, c->part_hist, hn * 8)) || (s = ensure(c, c->part_base, hn * 8)) ||
            (s = ensure(c, c->part_tmp, scan_tmp_elems(hn) * 8)))
            return s;
        const uint64_t ng = nr * G;
        if (pre0 < 0 && ((s = ensure(c, c->part_codes, ng * 4 + 16)) || (s = ensure(c, c->part_inval, ng * 2 + 16))))
            return s;
        if (pre0 < 0) {  // (buffers may have moved)
            l.codes = (const uint32_t*)c->part_codes.p;
            l.inval = (const uint16_t*)c->part_inval.p;
        }
        // this pass's P2 output: keys_a (+ digs), or fin_packed when the
        // previous pass's walk wrote it (two passes per walk)
        const bool from_u = kpass && kp_u_pass == kpi;
        uint64_t* p2_keys = from_u ? kp_u_keys : c->keys_a;
        const uint64_t p2_stride = from_u ? kp_u_n : c->key_cap;
        const uint8_t* p2_digs = from_u ? (const uint8_t*)(kp_u_keys + (size_t)W * kp_u_n) : c->digs;
        const uint64_t* p2_base = (const uint64_t*)(from_u ? c->part_base2.p : c->part_base.p);
        uint64_t n = from_u ? kp_u_n : 0;
        if (!from_u) {
            // (the second pass's keys are read by the regional scatter only:
            // builds whose P3 tile differs from its tile take p3_scatter_k)
            const bool dual = kpass && kp_direct && kpi + 2 < kp.size() && !test_hook("KC_NO_DUAL_PASS") &&
                              !test_hook("KC_P3_SCATTER") && p3_tile(W) == rp_tile(W, false);
            if (dual && (s = ensure(c, c->part_base2, hn * 8))) return s;
            HIPCHK(c, hipEventRecord(c->ev0, c->stream));
            if (pre0 < 0)
                HIPCHK(c, launch_encode_reads(l, (uint32_t*)c->part_codes.p, (uint16_t*)c->part_inval.p, c->stream));
            if (kpass)  // the pass's histogram from the planner's grouped one (no walk)
                HIPCHK(c, launch_hist_group_sum((const uint64_t*)c->part_ghist.p, pg.nseg, l.flo / 16, l.fhi / 16,
                                                (uint64_t*)c->part_hist.p, c->stream));
            else
                HIPCHK(c, launch_part_hist(l, pg, (uint64_t*)c->part_hist.p, 48, c->stream));
            HIPCHK(c, launch_scan_u64((uint64_t*)c->part_hist.p, (uint64_t*)c->part_base.p, hn,
                                      (uint64_t*)c->part_tmp.p, c->stream));
            uint64_t tail[4] = {0, 0, 0, 0};
            HIPCHK(c, hipMemcpyAsync(&tail[0], (uint64_t*)c->part_base.p + hn - 1, 8, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipMemcpyAsync(&tail[1], (uint64_t*)c->part_hist.p + hn - 1, 8, hipMemcpyDeviceToHost, c->stream));
            if (dual) {
                HIPCHK(c, launch_hist_group_sum((const uint64_t*)c->part_ghist.p, pg.nseg, kp[kpi + 1] / 16,
                                                kp[kpi + 2] / 16, (uint64_t*)c->part_hist.p, c->stream));
                HIPCHK(c, launch_scan_u64((uint64_t*)c->part_hist.p, (uint64_t*)c->part_base2.p, hn,
                                          (uint64_t*)c->part_tmp.p, c->stream));
                HIPCHK(c, hipMemcpyAsync(&tail[2], (uint64_t*)c->part_base2.p + hn - 1, 8, hipMemcpyDeviceToHost,
                                         c->stream));
                HIPCHK(c, hipMemcpyAsync(&tail[3], (uint64_t*)c->part_hist.p + hn - 1, 8, hipMemcpyDeviceToHost,
                                         c->stream));
            }
            HIPCHK(c, hipEventRecord(c->ev1, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
            c->part_ms[0] += t;
            n = tail[0] + tail[1];
            if (n > c->key_cap)
                return fail(c, KC_ERR_INTERNAL, "batch keys %llu exceed capacity", (unsigned long long)n);
            // the second pass's keys go past the records this pass will write
            // (key 0 slot + the earlier passes' records + this pass's keys)
            uint64_t* u = nullptr;
            const uint64_t n2 = tail[2] + tail[3];
            if (dual) {
                const size_t at = ((1 + kp_out + n) * (size_t)c->rs + 15) & ~(size_t)15;
                if (at + n2 * (8 * (size_t)W + 1) <= c->fin_packed.bytes && n2 > 0)
                    u = (uint64_t*)((uint8_t*)c->fin_packed.p + at);
            }
            if (u) {
                l.fhi = kp[kpi + 2];  // the walk keeps both passes' ranges
            }
            HIPCHK(c, hipEventRecord(c->ev0, c->stream));
            // (p2_no_digs: P2 writes no digit bytes, P3's histogram reads word 0)
            HIPCHK(c, launch_part_scatter(l, pg, (const uint64_t*)c->part_base.p, c->keys_a, c->key_cap, 48,
                                          p2_no_digs ? nullptr : c->digs, c->stream,
                                          u ? (const uint64_t*)c->part_base2.p : nullptr, u, u ? n2 : 0,
                                          u && !p2_no_digs ? (uint8_t*)(u + (size_t)W * n2) : nullptr,
                                          u ? kp[kpi + 1] : 256u, p2_aos));
            HIPCHK(c, hipEventRecord(c->ev1, c->stream));
            HIPCHK(c, hipEventSynchronize(c->ev1));
            HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
            c->part_ms[1] += t;
            c->st.insert_launches++;
            c->st.insert_ms += t;
            if (u) {
                kp_u_pass = kpi + 1;
                kp_u_keys = u;
                kp_u_n = n2;
            }
        }

        if (experiment_knob("KC_P2_SKIP")) {  // keys are invalid, stop after P2
            c->batches++;
            done += nr;
            continue;
        }
        if (n > 0) {
            // P3 tiles: regions (P2 digits) cut into tiles of their own
            std::vector<uint64_t> rt(2 * 257);
            HIPCHK(c, hipMemcpy2DAsync(rt.data(), 8, p2_base, pg.nseg * 8, 8, 256, hipMemcpyDeviceToHost,
                                       c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            rt[256] = n;
            const uint64_t tile = (uint64_t)p3_tile(W);
            rt[257] = 0;
            for (int r = 0; r < 256; r++) rt[257 + r + 1] = rt[257 + r] + (rt[r + 1] - rt[r] + tile - 1) / tile;
            const uint64_t ntiles = rt[257 + 256];
            if ((s = ensure(c, c->part_sort_hist, (256 * ntiles + p3_tmp_elems(ntiles) + 2 * 257) * 8))) return s;
            uint64_t* p3h = (uint64_t*)c->part_sort_hist.p;
            uint64_t* p3t = p3h + 256 * ntiles + p3_tmp_elems(ntiles);
            HIPCHK(c, hipMemcpyAsync(p3t, rt.data(), 2 * 257 * 8, hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipEventRecord(c->ev0, c->stream));
            if (p2_no_digs)
                HIPCHK(c, launch_rp_hist(nullptr, p2_keys, 56, p3t, p3t + 257, 256, ntiles, (uint32_t)tile, p3h,
                                         p3h + 256 * ntiles, 2 * c->n_cu, c->stream));
            else
                HIPCHK(c, launch_p3_hist(W, p2_digs, p3t, p3t + 257, ntiles, p3h, p3h + 256 * ntiles, 2 * c->n_cu,
                                         c->stream));
            HIPCHK(c, hipEventRecord(c->ev1, c->stream));
            HIPCHK(c, hipEventSynchronize(c->ev1));
            HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
            c->part_ms[3] += t;
            HIPCHK(c, hipEventRecord(c->ev0, c->stream));
            uint8_t* p3b_digs = nullptr;  // P3b digit bytes written by P3 (else P3b reads word 0)
            bool p3_aos = false;          // P3's output keys AoS (only when P3b follows)
            bool p3b_aos = false;         // P3b's output keys AoS
            // decided once: P3's output layout and P5's input depend on it
            const bool p3b = c->hc_hint && n >= p3b_min_of() && !test_hook("KC_NO_P3B");
            // P3's scatter is the regional radix scatter (digit word0 >> 56 over
            // the 256 P2 regions, same tiles; next tile's run starts prefetched,
            // XCD-aware tile walk); KC_P3_SCATTER: the older p3_scatter_k
            if (test_hook("KC_P3_SCATTER") || p3_tile(W) != rp_tile(W, false)) {
                if (from_u) return fail(c, KC_ERR_INTERNAL, "p3_scatter_k reads keys_a only");
                HIPCHK(c, launch_p3_scatter(W, c->keys_a, c->keys_b, c->key_cap, p3t, p3t + 257, ntiles, p3h,
                                            2 * c->n_cu, c->stream));
            } else {
                // a P3b pass follows (high cardinality): P3 writes each key's P3b
                // digit byte (bits 40..47) into the free P2 digit array, so P3b's
                // histogram reads 1 B per key, not word 0
                p3b_digs = p3b ? c->digs : nullptr;
                // ... and writes the keys AoS for it (P3b reads them so)
                p3_aos = p3b_digs && !test_hook("KC_P3_SOA");
                HIPCHK(c, launch_rp_scatter(W, false, p2_keys, p2_aos ? 0 : p2_stride, c->keys_b,
                                            p3_aos ? 0 : c->key_cap, nullptr, nullptr, p3t, p3t + 257, 256, ntiles,
                                            p3h, 56, p3b_digs, 40, 2 * c->n_cu, c->stream));
            }
            HIPCHK(c, hipEventRecord(c->ev1, c->stream));
            HIPCHK(c, hipEventSynchronize(c->ev1));
            HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
            c->part_ms[2] += t;
            c->part_keys += n;

            uint32_t nb = 1u << kBucketBits;
            if ((s = ensure(c, c->part_starts, ((size_t)nb + 1) * 8))) return s;
            HIPCHK(c, hipEventRecord(c->ev0, c->stream));
            HIPCHK(c, launch_bucket_bounds(W, c->keys_b, p3_aos ? 0 : c->key_cap, n, kBucketBits,
                                           (uint64_t*)c->part_starts.p, c->stream));
            HIPCHK(c, hipEventRecord(c->ev1, c->stream));
            HIPCHK(c, hipEventSynchronize(c->ev1));
            HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
            c->part_ms[3] += t;

            // P3b (high cardinality: most keys distinct): every bucket split
            // once more by key bits 40..47 (a regional radix pass keys_b ->
            // keys_a over the 65536 buckets), so P5 counts runs of
            // consecutive sub-buckets in one pass each and reads every key
            // once instead of once per sub-range pass
            uint64_t* p5_keys = c->keys_b;
            uint64_t p5_stride = p3_aos ? 0 : c->key_cap;  // 0: AoS (P3's or P3b's output)
            uint64_t* p5_spill = c->keys_a;
            const uint64_t* sub_starts = nullptr;
            if (p3b) {
                // P3's AoS output always comes with its digit bytes (the
                // regional histogram reads word 0 from SoA keys only)
                if (p3_aos && !p3b_digs) return fail(c, KC_ERR_INTERNAL, "P3b: AoS keys without digit bytes");
                std::vector<uint64_t> rs((size_t)nb + 1);
                HIPCHK(c, hipMemcpyAsync(rs.data(), c->part_starts.p, rs.size() * 8, hipMemcpyDeviceToHost, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
                const uint64_t tile = (uint64_t)rp_tile(W, false);
                std::vector<uint64_t> rt(2 * ((size_t)nb + 1));
                for (uint32_t r = 0; r <= nb; r++) rt[r] = rs[r];
                uint64_t* tp = rt.data() + nb + 1;
                tp[0] = 0;
                for (uint32_t r = 0; r < nb; r++) tp[r + 1] = tp[r] + (rs[r + 1] - rs[r] + tile - 1) / tile;
                const uint64_t nt = tp[nb];
                const size_t pos_n = 256 * nt, cnt_n = (256 * nt + 1) / 2;
                if ((s = ensure(c, c->p3b_buf, (pos_n + cnt_n + rt.size()) * 8)) ||
                    (s = ensure(c, c->sub_starts, (((size_t)nb << 8) + 1) * 8)))
                    return s;
                uint64_t* pos = (uint64_t*)c->p3b_buf.p;
                uint32_t* cnt_t = (uint32_t*)(pos + pos_n);
                uint64_t* rtd = pos + pos_n + cnt_n;
                HIPCHK(c, hipMemcpyAsync(rtd, rt.data(), rt.size() * 8, hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipEventRecord(c->ev0, c->stream));
                HIPCHK(c, launch_rp_hist_regional(c->keys_b, 40, rtd, rtd + nb + 1, (int)nb, nt, (uint32_t)tile, pos,
                                                  cnt_t, 2 * c->n_cu, c->stream, p3b_digs));
                // (its output AoS too, for P5s / the hash path; KC_P3B_SOA: arrays)
                p3b_aos = !test_hook("KC_P3B_SOA");
                HIPCHK(c, launch_rp_scatter(W, false, c->keys_b, p3_aos ? 0 : c->key_cap, c->keys_a,
                                            p3b_aos ? 0 : c->key_cap, nullptr, nullptr,
                                            rtd, rtd + nb + 1, (int)nb, nt, pos, 40, nullptr, 0, 2 * c->n_cu,
                                            c->stream));
                HIPCHK(c, launch_sub_starts(rtd, rtd + nb + 1, pos, nb, n, (uint64_t*)c->sub_starts.p, c->stream));
                HIPCHK(c, hipEventRecord(c->ev1, c->stream));
                HIPCHK(c, hipEventSynchronize(c->ev1));
                HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
                c->part_ms[2] += t;
                c->presplit_ms += t;
                c->presplit_batches++;
                p5_keys = c->keys_a;
                p5_stride = p3b_aos ? 0 : c->key_cap;
                p5_spill = c->keys_b;
                sub_starts = (const uint64_t*)c->sub_starts.p;
            }

            // Records: at most one LDS table per bucket unless buckets were
            // split into sub-range passes (high cardinality); on overflow P5
            // reruns with a bigger buffer (safe while nothing went to the
            // fallback table or the spill, whose inserts are not idempotent).
            uint64_t lslots = (uint64_t)bucket_lds_slots(W);
            uint64_t bound = (uint64_t)nb * lslots;
            if (bound > n || c->hc_hint) bound = n;  // high cardinality: about one record per key
            const uint64_t rec0 = c->rec_n;
            const uint64_t claimed0 = c->stats_h[ST_CLAIMED];
            const uint64_t desc0 = c->stats_h[ST_DESC_FILL];
            if ((s = ensure(c, c->desc_key, kDescCap * 8)) || (s = ensure(c, c->desc_start, kDescCap * 8)) ||
                (s = ensure(c, c->desc_len, kDescCap * 4)))
                return s;
            // P5s: pre-split runs sorted in LDS (records <= keys, no overflow);
            // the runs it flags (a sub-bucket too big, clustered keys) take
            // the LDS hash table (KC_NO_SORT_RUNS: hash table for all runs)
            const bool sort_runs = sub_starts && !test_hook("KC_NO_SORT_RUNS");
            uint64_t direct_min = 1ull << 22;  // (KC_P5S_DIRECT_MIN: path selector for tests)
            if (const char* e = test_hook("KC_P5S_DIRECT_MIN")) direct_min = strtoull(e, nullptr, 10);
            if (kpass && kp_direct) {
                // key-range pass: appended to the direct run of the earlier passes
                bool dd = false;
                uint64_t R = 0;
                float t5 = 0.f;
                const bool last = kpi + 2 == kp.size();
                if (sort_runs) {
                    const size_t fl = ((size_t)nb << 8) + nb + 16;
                    if ((s = ensure(c, c->run_flags, fl))) return s;
                    if ((s = p5s_direct(c, p5_keys, p5_stride, sub_starts, nb, n, (uint8_t*)c->run_flags.p, fl, &dd, &R, &t5,
                                        kp_out, kp_keys, last)))
                        return s;
                    c->part_ms[4] += t5;
                    c->p5_launches++;
                    if (getenv("KC_DEBUG"))
                        fprintf(stderr, "kc: P5s direct pass %zu [%u, %u) n=%llu records=%llu kept=%d %.3f ms\n", kpi,
                                kp[kpi], kp[kpi + 1], (unsigned long long)n, (unsigned long long)R, dd ? 1 : 0, t5);
                }
                if (dd) {
                    kp_out += R;
                    c->engines_used |= 2u;
                    if (!last) {
                        kpi++;
                        continue;
                    }
                    c->sorted_run_batches++;
                    done += nr;
                    continue;
                }
                // this pass cannot go direct: the earlier passes become a
                // finished run, this pass and the later ones count into records
                kp_direct = false;
                if (kp_out > 0 && (s = direct_keep(c, kp_out))) return s;
            }
            if (!kpass && sort_runs && c->rec_n == 0 && c->batches == 0 && c->stats_h[ST_CLAIMED] == 0 && !c->skm_used &&
                c->runs.empty() && n >= direct_min && !test_hook("KC_NO_P5S_DIRECT")) {
                const size_t fl = ((size_t)nb << 8) + nb + 16;
                if ((s = ensure(c, c->run_flags, fl))) return s;
                bool dd = false;
                uint64_t R = 0;
                float t5 = 0.f;
                if ((s = p5s_direct(c, p5_keys, p5_stride, sub_starts, nb, n, (uint8_t*)c->run_flags.p, fl, &dd, &R, &t5)))
                    return s;
                c->part_ms[4] += t5;
                c->p5_launches++;
                if (getenv("KC_DEBUG"))
                    fprintf(stderr, "kc: P5s direct n=%llu records=%llu kept=%d %.3f ms\n", (unsigned long long)n,
                            (unsigned long long)R, dd ? 1 : 0, t5);
                if (dd) {
                    c->sorted_run_batches++;
                    c->hc_hint = R * 2 > n;
                    c->engines_used |= 2u;
                    done += nr;
                    continue;
                }
            }
            if (sort_runs) {
                if ((s = grow_records(c, rec0 + n))) return s;
                const size_t fl = ((size_t)nb << 8) + nb + 16;
                if ((s = ensure(c, c->run_flags, fl))) return s;
                uint8_t* rf = (uint8_t*)c->run_flags.p;
                uint8_t* bf = rf + ((size_t)nb << 8);
                uint32_t* nflag = (uint32_t*)(bf + nb);
                HIPCHK(c, hipMemsetAsync(rf, 0, fl, c->stream));
                HIPCHK(c, hipEventRecord(c->ev0, c->stream));
                HIPCHK(c, launch_sort_runs(W, p5_keys, p5_stride, sub_starts, nb, c->rec_keys, c->rec_cnts,
                                           c->rec_cap, c->rec_cursor, c->stats, (uint64_t*)c->desc_key.p,
                                           (uint64_t*)c->desc_start.p, (uint32_t*)c->desc_len.p, kDescCap, rf, bf,
                                           nflag, 2 * c->n_cu, c->stream));
                uint32_t nf = 0;
                HIPCHK(c, hipMemcpyAsync(&nf, nflag, 4, hipMemcpyDeviceToHost, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
                if (nf)
                    HIPCHK(c, launch_count_buckets(W, p5_keys, p5_stride, (const uint64_t*)c->part_starts.p, nb,
                                                   c->rec_keys, c->rec_cnts, c->rec_cap, c->rec_cursor, c->table,
                                                   c->cap, p5_spill, c->key_cap, c->stats, l.probe_limit,
                                                   c->cfg.lds_slots, c->n_cu, (uint64_t*)c->desc_key.p,
                                                   (uint64_t*)c->desc_start.p, (uint32_t*)c->desc_len.p, kDescCap,
                                                   c->stream, true, sub_starts, rf, bf,
                                                   (uint32_t)sort_runs_keys(W)));
                HIPCHK(c, hipEventRecord(c->ev1, c->stream));
                HIPCHK(c, hipMemcpyAsync(&c->rec_n, c->rec_cursor, 8, hipMemcpyDeviceToHost, c->stream));
                if ((s = sync_stats(c))) return s;
                HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
                c->part_ms[4] += t;
                c->p5_launches++;
                c->sorted_run_batches++;
                if (getenv("KC_DEBUG"))
                    fprintf(stderr, "kc: P5s n=%llu runs=%llu flagged=%u records=%llu %.3f ms\n",
                            (unsigned long long)n, (unsigned long long)c->stats_h[ST_P5_PASSES], nf,
                            (unsigned long long)c->rec_n, t);
                if (c->stats_h[ST_ERR] & ERR_REC_OVERFLOW) return fail(c, KC_ERR_INTERNAL, "record buffer overflow");
            }
            for (; !sort_runs;) {
                if ((s = grow_records(c, rec0 + bound))) return s;
                // keys_a is free after P3: it takes P5's spills (capacity >= n)
                HIPCHK(c, hipEventRecord(c->ev0, c->stream));
                HIPCHK(c, launch_count_buckets(W, p5_keys, p5_stride, (const uint64_t*)c->part_starts.p, nb,
                                               c->rec_keys, c->rec_cnts, c->rec_cap, c->rec_cursor, c->table, c->cap,
                                               p5_spill, c->key_cap, c->stats, l.probe_limit, c->cfg.lds_slots,
                                               c->n_cu, (uint64_t*)c->desc_key.p, (uint64_t*)c->desc_start.p,
                                               (uint32_t*)c->desc_len.p, kDescCap, c->stream, c->hc_hint, sub_starts));
                HIPCHK(c, hipEventRecord(c->ev1, c->stream));
                HIPCHK(c, hipMemcpyAsync(&c->rec_n, c->rec_cursor, 8, hipMemcpyDeviceToHost, c->stream));
                if ((s = sync_stats(c))) return s;
                HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
                c->part_ms[4] += t;
                c->p5_launches++;
                if (getenv("KC_DEBUG"))
                    fprintf(stderr, "kc: P5 n=%llu passes=%llu aborts=%llu max_m=%llu records=%llu %.3f ms\n",
                            (unsigned long long)n, (unsigned long long)c->stats_h[ST_P5_PASSES],
                            (unsigned long long)c->stats_h[ST_P5_ABORTS], (unsigned long long)c->stats_h[ST_P5_MAXM],
                            (unsigned long long)c->rec_n, t);
                if (!(c->stats_h[ST_ERR] & ERR_REC_OVERFLOW)) break;
                if (bound >= n || c->stats_h[ST_CLAIMED] != claimed0 || c->stats_h[ST_SPILL2_FILL])
                    return fail(c, KC_ERR_INTERNAL, "record buffer overflow");
                bound = n;
                uint64_t err = c->stats_h[ST_ERR] & ~(uint64_t)ERR_REC_OVERFLOW;
                HIPCHK(c, hipMemcpyAsync(c->stats + ST_ERR, &err, 8, hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipMemcpyAsync(c->rec_cursor, &rec0, 8, hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipMemcpyAsync(c->stats + ST_DESC_FILL, &desc0, 8, hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
                c->stats_h[ST_DESC_FILL] = desc0;
                c->stats_h[ST_ERR] = err;
                c->rec_n = rec0;
            }
            // the next batch's P5 starts from this one's cardinality
            c->hc_hint = (c->rec_n - rec0) * 2 > n;
            if (c->stats_h[ST_ERR] & ERR_SPILL_OVERFLOW) return fail(c, KC_ERR_INTERNAL, "spill buffer overflow");
            uint64_t n2 = c->stats_h[ST_SPILL2_FILL];
            if (n2) {
                if ((s = flush_keys(c, p5_spill, c->key_cap, n2, p5_keys))) return s;
                HIPCHK(c, hipMemsetAsync(c->stats + ST_SPILL2_FILL, 0, 8, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
                c->stats_h[ST_SPILL2_FILL] = 0;
            }
        } else if ((s = sync_stats(c))) {
            return s;
        }
        c->batches++;
        c->engines_used |= 2u;
        // records past half the working set become a sorted run between
        // batches and between passes that did not go direct, as pend_flush
        // does between its calls (a call of many batches or passes must not
        // grow the records past the working set). Not while the next pass's
        // keys wait in fin_packed (two passes per walk), which the cut writes.
        if (!(kpass && kp_u_pass == kpi + 1) && (s = cut_run_if_full(c))) return s;
        if (kpass && kpi + 2 < kp.size()) {
            kpi++;
            continue;
        }
        done += nr;
    }
    c->st.valid_kmers = c->stats_h[ST_VALID];
    c->st.spilled_kmers = c->spilled_flushed + c->stats_h[ST_SPILL_FILL];
    return KC_OK;
}

// ---------------------------------------------------------------------------
// Engine "skm" (super-k-mer records; kernels and record layout in kc_skm.inl)
// ---------------------------------------------------------------------------

// Groups n SoA items (NW words at stride sa in `a`, optional u32 payload pa)
// by the 16 bits word0 >> 48: level 1 by bits 48..55 into `b` (writing the
// level-2 digit, bits 56..63, of every item to `digs`), level 2 by bits 56..63
// stable over level 1's regions, back into `a`. ms[0] += histogram + scan
// time, ms[1] += scatter time (HIP events).
static kc_status group16(kc_ctx* c, int NW, bool pay, uint64_t* a, uint64_t sa, uint32_t* pa, uint64_t* b,
                         uint64_t sb, uint32_t* pb, uint8_t* digs, uint64_t n, double* ms,
                         const uint8_t* dig1 = nullptr) {
    if (n == 0) return KC_OK;
    kc_status s;
    const uint64_t tile = (uint64_t)rp_tile(NW, pay);
    const uint64_t nt1 = (n + tile - 1) / tile;
    const uint64_t ntmax = nt1 + 256;
    const uint64_t tmpn = p3_tmp_elems(ntmax);
    if ((s = ensure(c, c->part_sort_hist, (256 * ntmax + tmpn + 4 + 2 * 257) * 8))) return s;
    uint64_t* pos = (uint64_t*)c->part_sort_hist.p;
    uint64_t* tmp = pos + 256 * ntmax;
    uint64_t* rt = tmp + tmpn;
    const int grid = 2 * c->n_cu;
    float t = 0.f;
    std::vector<uint64_t> h(4 + 2 * 257);
    h[0] = 0;
    h[1] = n;
    h[2] = 0;
    h[3] = nt1;
    HIPCHK(c, hipMemcpyAsync(rt, h.data(), 4 * 8, hipMemcpyHostToDevice, c->stream));
    // (histogram and scatter timed by three marks and the one synchronisation
    // each pass needs anyway: no wait between a histogram and its scatter)
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    // first pass digit: the producer's byte per item when it wrote one, else word 0 bits 48..55
    HIPCHK(c, launch_rp_hist(dig1, dig1 ? nullptr : a, 48, rt, rt + 2, 1, nt1, (uint32_t)tile, pos, tmp, grid,
                             c->stream));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, launch_rp_scatter(NW, pay, a, sa, b, sb, pa, pb, rt, rt + 2, 1, nt1, pos, 48, digs, 56, grid,
                                c->stream));
    HIPCHK(c, hipEventRecord(c->ev2, c->stream));
    std::vector<uint64_t> dbase(256);
    HIPCHK(c, hipMemcpyAsync(dbase.data(), rp_digit_base(tmp, nt1), 256 * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
    ms[0] += t;
    HIPCHK(c, hipEventElapsedTime(&t, c->ev1, c->ev2));
    ms[1] += t;
    uint64_t* rs = h.data() + 4;
    uint64_t* tp = rs + 257;
    for (int d = 0; d < 256; d++) rs[d] = dbase[d];
    rs[256] = n;
    tp[0] = 0;
    for (int d = 0; d < 256; d++) tp[d + 1] = tp[d] + (rs[d + 1] - rs[d] + tile - 1) / tile;
    const uint64_t nt2 = tp[256];
    HIPCHK(c, hipMemcpyAsync(rt + 4, rs, 2 * 257 * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, launch_rp_hist(digs, nullptr, 0, rt + 4, rt + 4 + 257, 256, nt2, (uint32_t)tile, pos, tmp, grid,
                             c->stream));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, launch_rp_scatter(NW, pay, b, sb, a, sa, pb, pa, rt + 4, rt + 4 + 257, 256, nt2, pos, 56, nullptr, 0,
                                grid, c->stream));
    HIPCHK(c, hipEventRecord(c->ev2, c->stream));
    HIPCHK(c, hipEventSynchronize(c->ev2));
    HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
    ms[0] += t;
    HIPCHK(c, hipEventElapsedTime(&t, c->ev1, c->ev2));
    ms[1] += t;
    return KC_OK;
}

// Reads of nw windows one skm batch may take beyond key_cap windows (see
// count_reads_skm): the record pool at nw / 4 records per read, while the
// global table is empty; 0 when only safe batches apply
static uint64_t skm_big_reads(const kc_ctx* c, uint64_t nw, uint64_t pool_cap) {
    if (c->skm_big_off || c->stats_h[ST_CLAIMED] || c->table_dirty || test_hook("KC_SKM_SAFE_BATCH")) return 0;
    return pool_cap / std::max<uint64_t>(1, nw / 4);
}

// part_ms slots for this engine: [0] E + F, [1] F, [2] S1/S2 scatters,
// [3] S1/S2 histograms + scans + P4, [4] P5.
static kc_status count_reads_skm(kc_ctx* c, const uint8_t* base, const uint64_t* seq_off, uint64_t n_reads,
                                 int64_t L, const SkmGeom& g, int64_t pre0) {
    if (c->finished) return fail(c, KC_ERR_STATE, "kc_finish was called; kc_reset first");
    const int W = c->W;
    const int RW = W + 1;
    const uint64_t nw = (uint64_t)(L - c->k + 1);
    // keys_a / keys_b hold RW x pool_cap record words each; digs holds a byte per record
    uint64_t pool_cap = (uint64_t)W * c->key_cap / RW;
    if (const char* e = test_hook("KC_SKM_POOL_CAP")) {  // tests: force the pool-overflow retry
        const uint64_t v = strtoull(e, nullptr, 10);
        if (v > 0 && v < pool_cap) pool_cap = v;
    }
    // P5's spills go to keys_b (key_cap keys), which a batch of at most
    // key_cap windows can never overflow. While the global table is still
    // empty a batch may be larger, up to what the record pool holds at nw / 4
    // records per read (F's pool-overflow retry catches denser reads): fewer
    // batches, so fewer runs for the finish to merge (SURVEY cfg4: 125M reads
    // per GPU in one batch). A spill overflow in such a batch undoes it (table
    // cleared, records and statistics restored) and retries it at the safe size.
    uint64_t safe_reads = c->key_cap / nw;
    if (safe_reads == 0) return fail(c, KC_ERR_ARG, "gpu_memory_limit too small for one read's windows");
    uint64_t max_reads = std::max(safe_reads, skm_big_reads(c, nw, pool_cap));
    // even batch sizes when a read's code row is an odd number of words: every
    // batch's masks then start 4-byte aligned, which F3's dword DMA needs
    const bool even = (groups_per_read((int)L) & 1) != 0;
    auto even_down = [&](uint64_t v) { return even && v > 1 ? v & ~1ull : v; };
    safe_reads = even_down(safe_reads);
    max_reads = even_down(max_reads);
    kc_status s;
    uint64_t done = 0;
    float t = 0.f;
    while (done < n_reads) {
        uint64_t nr = n_reads - done;
        if (nr > max_reads) nr = max_reads;
        if (nr > safe_reads && (c->stats_h[ST_CLAIMED] || c->table_dirty)) {
            nr = safe_reads;  // the table holds keys already: only a safe batch
            max_reads = safe_reads;
        }
        const bool big = nr > safe_reads;
        CountLaunch l;
        l.base = base;
        l.seq_off = seq_off;
        l.read0 = done;
        l.n_reads = nr;
        l.L = (int)L;
        l.k = (int)c->k;
        l.table = c->table;
        l.cap = c->cap;
        l.spill = c->spill;
        l.spill_cap = c->spill_cap;
        l.stats = c->stats;
        l.probe_limit = probe_limit(c);
        const uint64_t G = (uint64_t)groups_per_read((int)L);
        const uint64_t ng = nr * G;
        if (pre0 < 0 && ((s = ensure(c, c->part_codes, ng * 4 + 16)) || (s = ensure(c, c->part_inval, ng * 2 + 16))))
            return s;
        const uint64_t g0 = pre0 < 0 ? 0 : ((uint64_t)pre0 + done) * G;
        l.codes = (const uint32_t*)c->part_codes.p + g0;
        l.inval = (const uint16_t*)c->part_inval.p + g0;
        l.rlen = (pre0 >= 0 && c->var_rlen) ? c->var_rlen + (uint64_t)pre0 + done : nullptr;
        if ((s = sync_stats(c))) return s;
        std::vector<uint64_t> saved(c->stats_h, c->stats_h + ST_N);
        // host-side counters of the batch, restored with the device ones when
        // the batch is undone (so kc_stats describes only the work kept)
        const HostCounters hsaved = host_counters(c);
        HIPCHK(c, hipMemsetAsync(c->pool_cursor, 0, 8, c->stream));
        HIPCHK(c, hipEventRecord(c->ev0, c->stream));
        if (pre0 < 0)
            HIPCHK(c, launch_encode_reads(l, (uint32_t*)c->part_codes.p, (uint16_t*)c->part_inval.p, c->stream));
        HIPCHK(c, hipEventRecord(c->ev1, c->stream));
        HIPCHK(c, hipEventSynchronize(c->ev1));
        HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
        c->part_ms[0] += t;
        HIPCHK(c, hipEventRecord(c->ev0, c->stream));
        // digs: the second array (16-byte aligned, for the histogram's 16-byte
        // loads) takes F's first-pass digits, the first the second pass's
        // (written by the first pass)
        const uint64_t dig1_off = (pool_cap + 15) & ~15ull;
        uint8_t* dig1 = dig1_off + pool_cap <= c->digs_bytes ? c->digs + dig1_off : nullptr;
        HIPCHK(c, launch_skm_front(l, g, c->keys_a, pool_cap, c->pool_cursor, 8 * c->n_cu, c->stream, dig1));
        HIPCHK(c, hipEventRecord(c->ev1, c->stream));
        uint64_t np = 0;
        HIPCHK(c, hipMemcpyAsync(&np, c->pool_cursor, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
        c->part_ms[0] += t;
        c->part_ms[1] += t;
        c->st.insert_launches++;
        c->st.insert_ms += t;
        if (np > pool_cap) {
            // more records than the pool holds (runs far shorter than usual):
            // undo the batch's statistics and retry with half the reads
            HIPCHK(c, hipMemcpyAsync(c->stats, saved.data(), ST_N * 8, hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            memcpy(c->stats_h, saved.data(), ST_N * 8);
            restore_host_counters(c, hsaved);
            if (nr <= 1) return fail(c, KC_ERR_INTERNAL, "skm pool overflow on one read");
            max_reads = nr / 2 > 1 ? even_down(nr / 2) : 1;
            continue;
        }
        if (experiment_knob("KC_F_SKIP")) {  // records are invalid, stop after F
            c->batches++;
            done += nr;
            continue;
        }
        if (np > 0) {
            double gm[2] = {0, 0};
            // S's scratch (the first pass's output) at the end of keys_b, at
            // the records' own stride: the radix scatter writes the start of
            // a large allocation ~25% slower than its end in every process
            // measured (tools/rp_bench)
            uint64_t* sbase = c->keys_b;
            uint64_t sbs = pool_cap;
            const uint64_t cs = (np + 255) & ~255ull;
            const uint64_t belems = (uint64_t)RW * pool_cap;
            if ((uint64_t)RW * cs <= belems && !test_hook("KC_S_SCRATCH_START")) {
                sbs = cs;
                sbase = c->keys_b + ((belems - (uint64_t)RW * cs) & ~255ull);
            }
            if ((s = group16(c, RW, false, c->keys_a, pool_cap, nullptr, sbase, sbs, nullptr, c->digs, np, gm,
                             dig1)))
                return s;
            c->part_ms[3] += gm[0];
            c->part_ms[2] += gm[1];
            c->part_keys += np;
            const uint32_t nb = 1u << kBucketBits;
            if ((s = ensure(c, c->part_starts, ((size_t)nb + 1) * 8))) return s;
            HIPCHK(c, hipEventRecord(c->ev0, c->stream));
            HIPCHK(c, launch_bucket_bounds(1, c->keys_a, pool_cap, np, kBucketBits, (uint64_t*)c->part_starts.p,
                                           c->stream));
            HIPCHK(c, hipEventRecord(c->ev1, c->stream));
            HIPCHK(c, hipEventSynchronize(c->ev1));
            HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
            c->part_ms[3] += t;
            const uint64_t kbound = nr * nw;
            const uint64_t rec_batch0 = c->rec_n;
            // P5a (W = 1): each bucket's distinct records written back over
            // the front of its range, multiplicities into the digit bytes
            // (free after S2, read as u32 indexed like the pool); P5 walks them
            SkmDedup dd = {};
            const bool dedup = W == 1 && !test_hook("KC_NO_DEDUP") && np <= c->digs_bytes / 4;
            // P5a's overflow lists (buckets whose distinct records overflow its
            // LDS table, deduplicated again in hash-split passes) go to the
            // pool's free tail: records [np, limit) of keys_a, their
            // multiplicities at the same indices of the digit-byte buffer (u32)
            const uint64_t over0 = (np + 63) & ~63ull;
            uint64_t over_limit = std::min<uint64_t>(pool_cap, c->digs_bytes / 4);
            if (const char* e = test_hook("KC_P5A_OVER_ROOM"))  // tests: little room, later buckets stay raw
                over_limit = std::min<uint64_t>(over_limit, over0 + strtoull(e, nullptr, 10));
            const size_t dpos_off = (((size_t)nb + 1) * 4 + 64 + 15) & ~(size_t)15;
            if (dedup) {
                if ((s = ensure(c, c->part_dedup, dpos_off + (size_t)nb * 8))) return s;
                dd.cnt = (const uint32_t*)c->digs;
                dd.len = (const uint32_t*)c->part_dedup.p;
                dd.pos = (const uint64_t*)((const uint8_t*)c->part_dedup.p + dpos_off);
                HIPCHK(c, hipMemcpyAsync(c->pool_cursor, &over0, 8, hipMemcpyHostToDevice, c->stream));
            }
            // P5 over buckets [b0, b1); reruns with a bigger record buffer on
            // overflow (safe while nothing went to the global table or spill).
            // A large batch (more than key_cap windows) does not grow the
            // buffer to its window count, which can be far past the working
            // set: it sets rec_retry, and the batch is undone and counted in
            // safe batches like a spill overflow
            bool rec_retry = false;
            auto p5_range = [&](uint32_t b0, uint32_t b1, bool count_keys) -> kc_status {
                uint64_t bound = (uint64_t)(b1 - b0) * (uint64_t)skm_lds_slots(W);
                if (bound > kbound) bound = kbound;
                if (const char* e = test_hook("KC_P5_REC_BOUND")) {  // tests: force the overflow path
                    const uint64_t v = strtoull(e, nullptr, 10);
                    if (v > 0 && v < bound) bound = v;
                }
                const uint64_t rec0 = c->rec_n;
                const uint64_t claimed0 = c->stats_h[ST_CLAIMED];
                kc_status s2;
                // P5a and P5 back to back, timed by three marks after P5's
                // synchronisation (P5a's time: ev0 -> ev1, P5's: ev1 -> ev2)
                bool p5a_pending = false;
                if (dedup) {
                    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
                    HIPCHK(c, launch_count_rec(c->keys_a, pool_cap, (const uint64_t*)c->part_starts.p, b0, b1,
                                               (uint32_t*)c->digs, (uint32_t*)c->part_dedup.p, c->n_cu, c->stream,
                                               over0 < over_limit ? c->pool_cursor : nullptr, over_limit,
                                               (uint64_t*)dd.pos));
                    p5a_pending = true;
                }
                for (;;) {
                    if ((s2 = grow_records(c, rec0 + bound))) return s2;
                    // keys_b is free after S2: it takes P5's spills (W x key_cap words)
                    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
                    HIPCHK(c, launch_count_skm(W, (int)c->k, c->keys_a, pool_cap, (const uint64_t*)c->part_starts.p,
                                               b0, b1, count_keys, c->rec_keys, c->rec_cnts, c->rec_cap,
                                               c->rec_cursor, c->table, c->cap, c->keys_b, c->key_cap, c->stats,
                                               l.probe_limit, c->cfg.lds_slots, c->n_cu, c->stream,
                                               dedup ? &dd : nullptr, c->rec_dig));
                    HIPCHK(c, hipEventRecord(c->ev2, c->stream));
                    HIPCHK(c, hipMemcpyAsync(&c->rec_n, c->rec_cursor, 8, hipMemcpyDeviceToHost, c->stream));
                    if ((s2 = sync_stats(c))) return s2;
                    if (p5a_pending) {
                        HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
                        c->dedup_ms += t;
                        p5a_pending = false;
                    }
                    HIPCHK(c, hipEventElapsedTime(&t, c->ev1, c->ev2));
                    c->part_ms[4] += t;
                    c->p5_launches++;
                    if (getenv("KC_DEBUG"))
                        fprintf(stderr,
                                "kc: skm F records=%llu P5[%u,%u) passes=%llu aborts=%llu max_m=%llu records=%llu %.3f ms\n",
                                (unsigned long long)np, b0, b1, (unsigned long long)c->stats_h[ST_P5_PASSES],
                                (unsigned long long)c->stats_h[ST_P5_ABORTS],
                                (unsigned long long)c->stats_h[ST_P5_MAXM], (unsigned long long)c->rec_n, t);
                    if (!(c->stats_h[ST_ERR] & ERR_REC_OVERFLOW)) return KC_OK;
                    if (big) {
                        rec_retry = true;
                        return KC_OK;
                    }
                    if (bound >= kbound || c->stats_h[ST_CLAIMED] != claimed0 || c->stats_h[ST_SPILL2_FILL])
                        return fail(c, KC_ERR_INTERNAL, "record buffer overflow");
                    bound = kbound;
                    uint64_t err = c->stats_h[ST_ERR] & ~(uint64_t)ERR_REC_OVERFLOW;
                    HIPCHK(c, hipMemcpyAsync(c->stats + ST_ERR, &err, 8, hipMemcpyHostToDevice, c->stream));
                    HIPCHK(c, hipMemcpyAsync(c->rec_cursor, &rec0, 8, hipMemcpyHostToDevice, c->stream));
                    HIPCHK(c, hipStreamSynchronize(c->stream));
                    c->stats_h[ST_ERR] = err;
                    c->rec_n = rec0;
                }
            };
            // bucket 0xffff holds only the pool's padding records. Unless this
            // context already knows its data, the first kSkmSample buckets are
            // counted alone: if most of their keys are distinct (iid reads, no
            // coverage) the key-prefix engine takes this batch and the rest,
            // whose sorted finish needs no global sort
            const uint32_t nbk = nb - 1;
            uint32_t bs = 0;
            if (!c->skm_force && !c->skm_checked && kbound >= kSkmSampleMinKeys) {
                bs = kSkmSample;
                if ((s = p5_range(0, bs, true))) return s;
                c->skm_checked = true;
                const uint64_t keys_s = c->stats_h[ST_P5_KEYS], dist_s = c->rec_n - rec_batch0;
                if (!rec_retry && keys_s > 0 && (double)dist_s > kSkmDistinctMax * (double)keys_s &&
                    c->stats_h[ST_CLAIMED] == saved[ST_CLAIMED] && c->stats_h[ST_SPILL2_FILL] == 0) {
                    HIPCHK(c, hipMemcpyAsync(c->stats, saved.data(), ST_N * 8, hipMemcpyHostToDevice, c->stream));
                    HIPCHK(c, hipMemcpyAsync(c->rec_cursor, &rec_batch0, 8, hipMemcpyHostToDevice, c->stream));
                    HIPCHK(c, hipStreamSynchronize(c->stream));
                    memcpy(c->stats_h, saved.data(), ST_N * 8);
                    c->rec_n = rec_batch0;
                    c->skm_hc = true;
                    c->hc_hint = true;
                    if (getenv("KC_DEBUG"))
                        fprintf(stderr, "kc: skm sample %llu distinct / %llu keys: key-prefix engine\n",
                                (unsigned long long)dist_s, (unsigned long long)keys_s);
                    return count_reads_part(c, seq_off ? base : base + done * (uint64_t)L,
                                            seq_off ? seq_off + done : nullptr, n_reads - done, L,
                                            pre0 < 0 ? -1 : pre0 + (int64_t)done);
                }
            }
            if (!rec_retry && (s = p5_range(bs, nbk, false))) return s;
            if (dedup && !rec_retry) {
                HIPCHK(c, launch_dedup_total((const uint32_t*)c->part_dedup.p, (const uint64_t*)c->part_starts.p, nbk,
                                             c->stats, c->stream));
                if ((s = sync_stats(c))) return s;
            }
            c->skm_used = true;
            c->engines_used |= 1u;
            if (((c->stats_h[ST_ERR] & ERR_SPILL_OVERFLOW) || rec_retry) && big) {
                // undo the large batch and count its reads in safe batches
                if (getenv("KC_DEBUG"))
                    fprintf(stderr, "kc: skm batch of %llu reads overflowed the %s buffer: retried\n",
                            (unsigned long long)nr, rec_retry ? "record" : "spill");
                HIPCHK(c, hipMemsetAsync(c->table, 0, c->table_bytes, c->stream));
                HIPCHK(c, hipMemcpyAsync(c->stats, saved.data(), ST_N * 8, hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipMemcpyAsync(c->rec_cursor, &rec_batch0, 8, hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
                memcpy(c->stats_h, saved.data(), ST_N * 8);
                restore_host_counters(c, hsaved);
                c->rec_n = rec_batch0;
                c->skm_big_off = true;
                max_reads = safe_reads;
                continue;
            }
            if (c->stats_h[ST_ERR] & ERR_SPILL_OVERFLOW) return fail(c, KC_ERR_INTERNAL, "spill buffer overflow");
            uint64_t n2 = c->stats_h[ST_SPILL2_FILL];
            if (n2) {
                if ((s = flush_keys(c, c->keys_b, c->key_cap, n2, c->keys_a))) return s;
                HIPCHK(c, hipMemsetAsync(c->stats + ST_SPILL2_FILL, 0, 8, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
                c->stats_h[ST_SPILL2_FILL] = 0;
            }
        } else if ((s = sync_stats(c))) {
            return s;
        }
        c->batches++;
        done += nr;
        // a call may span several batches (large batches, or safe ones once
        // the table holds keys): runs are cut between them as between calls
        if (done < n_reads && (s = cut_run_if_full(c))) return s;
    }
    c->st.valid_kmers = c->stats_h[ST_VALID];
    c->st.spilled_kmers = c->spilled_flushed + c->stats_h[ST_SPILL_FILL];
    return KC_OK;
}

// Engine choice before the super-k-mer engine's first large batch: the
// coverage sketch of the encoded reads (sketch_k). When most sampled k-mers
// are distinct (low coverage: iid reads, SURVEY cfg5) the key-prefix engine
// counts this batch and the rest of the context's input, and P5 splits its
// buckets up front; the super-k-mer engine's bucket sample (count_reads_skm)
// stays as the second check. Saves the skm engine's F and S passes over a
// batch it would give up.
static const double kSketchDistinctMax = 0.7;
static const double kSketchCoveredMax = 0.6;  // below: the skm bucket sample is not needed

static kc_status sketch_engine(kc_ctx* c, uint64_t n_reads, int64_t L, int64_t pre0) {
    kc_status s;
    const uint64_t G = (uint64_t)groups_per_read((int)L);
    // sample rate 2^-rb by k-mer hash: about 2^18 samples (at least 1/256)
    const uint64_t aligned = n_reads * G;
    int rb = 8;
    while (rb < 24 && (aligned >> rb) > (1ull << 18)) rb++;
    const uint64_t cap = (aligned >> rb) * 2 + 4096;  // twice the expected samples
    // the distinct samples are counted in a set of at least 2 x cap slots
    int set_bits = 1;
    while ((1ull << set_bits) < 2 * cap) set_bits++;
    const size_t set_bytes = ((size_t)8 << set_bits);
    if ((s = ensure(c, c->fin_keys[0], cap * 8 + 64)) || (s = ensure(c, c->fin_keys[1], set_bytes)) ||
        (s = ensure(c, c->fin_misc, 64)))
        return s;
    uint64_t* fp = (uint64_t*)c->fin_keys[0].p;
    uint64_t* counter = (uint64_t*)c->fin_misc.p;  // [0] samples, [1] distinct samples
    HIPCHK(c, hipMemsetAsync(counter, 0, 16, c->stream));
    HIPCHK(c, hipMemsetAsync(c->fin_keys[1].p, 0, set_bytes, c->stream));
    HIPCHK(c, launch_sketch((const uint32_t*)c->part_codes.p + (uint64_t)pre0 * G,
                            (const uint16_t*)c->part_inval.p + (uint64_t)pre0 * G, n_reads, (int)L, (int)c->k, rb, fp,
                            cap, counter, c->stream));
    HIPCHK(c, launch_sketch_distinct(fp, counter, cap, (uint64_t*)c->fin_keys[1].p, set_bits, counter + 1, c->stream));
    uint64_t md[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(md, counter, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    uint64_t m = md[0];
    if (m > cap) m = cap;
    if (m < 4096) return KC_OK;  // too few samples to tell: the skm engine's own sample decides
    const uint64_t distinct = md[1];
    if (getenv("KC_DEBUG"))
        fprintf(stderr, "kc: sketch %llu distinct / %llu sampled k-mers\n", (unsigned long long)distinct,
                (unsigned long long)m);
    if ((double)distinct > kSketchDistinctMax * (double)m) {
        c->skm_hc = true;
        c->hc_hint = true;
        c->skm_checked = true;
    } else if ((double)distinct < kSketchCoveredMax * (double)m && !test_hook("KC_SKM_SAMPLE")) {
        // clear coverage: the skm engine's bucket sample (its own check, at
        // 35% distinct keys) would keep the skm engine too; skipped, which
        // saves its two small launches and their synchronisation. (The sketch
        // samples only 16-base-aligned positions, so a k-mer covered c times
        // is sampled ~c/16 times: 60% distinct samples is a window coverage of
        // ~16, where about 6% of the keys are distinct)
        c->skm_checked = true;
    }
    return KC_OK;
}

// The coverage sketch picks the engine (auto) or, for the partition engine,
// sets the high-cardinality hint before its first batch
static kc_status sketch_gate(kc_ctx* c, uint64_t n_reads, int64_t L, int64_t pre0) {
    const bool skm_ok = skm_geometry((int)L, (int)c->k).ok;
    const bool sketch_skm = c->skm && !c->skm_hc && !c->skm_force && skm_ok;
    // (the key-prefix engine: chosen, or the default engine's only one for this (L, k))
    const bool sketch_part = c->part && !c->hc_hint && !(c->skm && !c->skm_hc && skm_ok);
    if ((sketch_skm || sketch_part) && !c->skm_checked && pre0 >= 0 && !test_hook("KC_NO_SKETCH") &&
        n_reads * (uint64_t)(L - c->k + 1) >= kSkmSampleMinKeys) {
        kc_status s = sketch_engine(c, n_reads, L, pre0);
        if (s) return s;
        if (sketch_part) c->skm_checked = true;  // once per reset
    }
    return KC_OK;
}

// pre0 >= 0: the reads are pre-encoded in part_codes / part_inval from read pre0
static kc_status count_reads(kc_ctx* c, const uint8_t* base, const uint64_t* seq_off, uint64_t n_reads, int64_t L,
                             int64_t pre0 = -1) {
    kc_status s0 = sketch_gate(c, n_reads, L, pre0);
    if (s0) return s0;
    // very long reads (one read's windows do not fit a P2 workgroup's LDS)
    // take the table engine; both feed the same finish
    if (c->skm && !c->skm_hc) {
        const SkmGeom g = skm_geometry((int)L, (int)c->k);
        if (g.ok) return count_reads_skm(c, base, seq_off, n_reads, L, g, pre0);
    }
    if (c->part && part_geometry((int)L, (int)c->k, 1).lds_scatter <= kMaxLds)
        return count_reads_part(c, base, seq_off, n_reads, L, pre0);
    if (pre0 >= 0) return fail(c, KC_ERR_INTERNAL, "pre-encoded reads reached the table engine");
    return count_reads_table(c, base, seq_off, n_reads, L);
}

// ---------------------------------------------------------------------------
// pending batch (see kc_ctx::pend_*)
// ---------------------------------------------------------------------------

// Reads of length L one engine batch holds (its window capacity key_cap)
static uint64_t batch_reads(const kc_ctx* c, int64_t L) {
    const uint64_t m = c->key_cap / (uint64_t)(L - c->k + 1);
    return m ? m : 1;
}

// Pending reads of length L allowed before a flush. While a checkpoint is held
// the batch may grow past one engine batch (count_reads splits it) up to
// 1/8 of the device's memory in codes (6 B per 16 bases), so a malformed block
// later in the same file can still be rolled back.
// Without a checkpoint the codes engines still pend up to 16 engine batches
// (within the same budget): a high-cardinality batch is then counted in
// key-range passes over all its reads instead of read batches whose runs must
// be merged (count_reads_part).
static uint64_t pend_room(const kc_ctx* c, int64_t L, bool var = false) {
    const uint64_t b = batch_reads(c, L);
    if (!c->ckpt && (!c->part || var)) return b;
    const uint64_t per_read = 6 * (uint64_t)groups_per_read((int)L) + 2;
    uint64_t budget = c->dev_total / 8 / per_read;
    if (!c->ckpt && budget / 16 > b) budget = 16 * b;
    return budget > b ? budget : b;
}

// Grows b to at least `bytes`, keeping its first `keep` bytes.
static kc_status grow_keep(kc_ctx* c, DevBuf& b, size_t bytes, size_t keep) {
    if (b.p && b.bytes >= bytes) return KC_OK;
    size_t want = bytes < 256 ? 256 : bytes;
    if (b.p && want < b.bytes + b.bytes / 2) want = b.bytes + b.bytes / 2;
    void* np = nullptr;
    HIPCHK(c, hipMalloc(&np, want));
    if (b.p && keep) HIPCHK(c, hipMemcpyAsync(np, b.p, keep, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (b.p) HIPCHK(c, hipFree(b.p));
    b.p = np;
    b.bytes = want;
    return KC_OK;
}

static kc_status cut_run_if_full(kc_ctx* c);

// Counts the pending batch (the engines: count_reads with pre-encoded reads).
extern "C" {
static kc_status chunk_acc_flush(kc_ctx* c);  // defined with the chunk entry points (C linkage block)
}

// Key 0's presence for reads whose slots hold positions that are no bases
// (variable-length padding, one-pass empty rows): the engines read those as
// not-ACGT, so it is recomputed as (presence before the flush) | ST_VHOLE (a
// read of >= k bases holds a not-ACGT base, set by the encoders) | a key-0
// window counted. Also applied before a run is cut inside such a flush.
static kc_status recompute_presence(kc_ctx* c) {
    kc_status s;
    if ((s = sync_stats(c))) return s;
    const uint64_t present =
        (c->flush_present0 | c->stats_h[ST_VHOLE] | (c->stats_h[ST_KEY0] != 0 ? 1u : 0u)) ? 1u : 0u;
    c->stats_h[ST_KEY0_PRESENT] = present;
    HIPCHK(c, hipMemcpyAsync(c->stats + ST_KEY0_PRESENT, &c->stats_h[ST_KEY0_PRESENT], 8, hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return KC_OK;
}

// Fixed-length pending reads [0, n): more than one engine batch is counted
// whole when it is a high-cardinality batch on an empty record state
// (key-range passes, count_reads_part), anything else batch by batch with a
// run cut between batches when the records outgrow half the working set
static kc_status pend_count_fixed(kc_ctx* c, uint64_t n) {
    kc_status s;
    const int64_t L = c->pend_L;
    const uint64_t b = batch_reads(c, L);
    if (n > b) {
        if ((s = sketch_gate(c, n, L, 0))) return s;
        const bool passes = c->hc_hint && c->part && (!c->skm || c->skm_hc) && c->rec_n == 0 && c->batches == 0 &&
                            !c->skm_used && c->runs.empty() && !test_hook("KC_NO_KEY_PASSES");
        if (!passes) {
            // the skm engine may take a large batch (count_reads_skm)
            uint64_t bs = b;
            if (c->skm && !c->skm_hc && skm_geometry((int)L, (int)c->k).ok) {
                const uint64_t nw = (uint64_t)(L - c->k + 1);
                bs = std::max(b, skm_big_reads(c, nw, (uint64_t)c->W * c->key_cap / (c->W + 1)));
            }
            // (an even read count per slice when a code row has an odd number
            // of words: each slice's masks start 4-byte aligned for F3)
            if ((groups_per_read((int)L) & 1) && bs > 1) bs &= ~1ull;
            for (uint64_t r0 = 0; r0 < n; r0 += bs) {
                if ((s = count_reads(c, nullptr, nullptr, n - r0 < bs ? n - r0 : bs, L, (int64_t)r0))) return s;
                if ((s = cut_run_if_full(c))) return s;
            }
            return KC_OK;
        }
    }
    if ((s = count_reads(c, nullptr, nullptr, n, L, 0))) return s;
    return cut_run_if_full(c);
}

static kc_status pend_flush(kc_ctx* c) {
    if (c->acc_n) {
        kc_status s0 = chunk_acc_flush(c);
        if (s0) return s0;
    }
    if (c->pend_reads == 0) return KC_OK;
    kc::trace("flush %llu reads of length %lld", (unsigned long long)c->pend_reads, (long long)c->pend_L);
    const uint64_t n = c->pend_reads;
    c->pend_reads = 0;  // a failed count is not counted again
    c->flushes++;
    const bool sparse = c->pend_sparse;
    c->pend_sparse = false;
    if (!c->pend_var && !sparse) return pend_count_fixed(c, n);
    // variable-length reads (slot padding) or one-pass rows (empty rows): the
    // skm front end reads each row's length; key 0's presence is recomputed
    kc_status s;
    if ((s = sync_stats(c))) return s;
    c->flush_present0 = c->stats_h[ST_KEY0_PRESENT];
    c->var_rlen = (const uint16_t*)c->part_rlen.p;
    s = c->pend_var ? count_reads(c, nullptr, nullptr, n, c->pend_L, 0) : pend_count_fixed(c, n);
    c->var_rlen = nullptr;
    if (s) return s;
    if ((s = recompute_presence(c))) return s;
    return c->pend_var ? cut_run_if_full(c) : KC_OK;
}

// Room for n_new more pending reads of length L (fixed or variable): the
// pending batch is counted first when it is of another kind or n_new would
// not fit; the buffers grow keeping the pending reads. *off receives the
// read index where the new reads go.
static kc_status pend_reserve(kc_ctx* c, int64_t L, bool var, uint64_t n_new, uint64_t* off, bool sparse = false) {
    kc_status s;
    if (c->pend_reads && (c->pend_L != L || c->pend_var != var || c->pend_reads + n_new > pend_room(c, L, var)))
        if ((s = pend_flush(c))) return s;
    const uint64_t G = (uint64_t)groups_per_read((int)L);
    const uint64_t keep = c->pend_reads * G, need = (c->pend_reads + n_new) * G;
    if ((s = grow_keep(c, c->part_codes, need * 4 + 16, keep * 4)) ||
        (s = grow_keep(c, c->part_inval, need * 2 + 16, keep * 2)))
        return s;
    if ((var || sparse || c->pend_sparse) &&
        (s = grow_keep(c, c->part_rlen, (c->pend_reads + n_new) * 2 + 16, c->pend_reads * 2)))
        return s;
    // a one-pass block joins reads of full length L: their lengths first
    if (sparse && !c->pend_sparse && c->pend_reads)
        HIPCHK(c, hipMemsetD16Async((hipDeviceptr_t)c->part_rlen.p, (unsigned short)L, c->pend_reads, c->stream));
    c->pend_L = L;
    c->pend_var = var;
    *off = c->pend_reads;
    return KC_OK;
}

// Encodes n_reads reads of device text into the pending batch, one engine
// batch at a time (kernel E): reads at r * L (reference chunks, seq_off null)
// or at seq_off[r] (variable-length: up to seq_end[r], padded slots).
static kc_status pend_add_reads(kc_ctx* c, const uint8_t* base, const uint64_t* seq_off, const uint64_t* seq_end,
                                uint64_t n_reads, int64_t L, bool var) {
    kc_status s;
    const uint64_t G = (uint64_t)groups_per_read((int)L);
    uint64_t done = 0;
    while (done < n_reads) {
        uint64_t free = 0;
        if (c->pend_L == L && c->pend_var == var && c->pend_reads < pend_room(c, L, var))
            free = pend_room(c, L, var) - c->pend_reads;
        if (free == 0 || c->pend_reads == 0) free = pend_room(c, L, var);
        const uint64_t m = n_reads - done < free ? n_reads - done : free;
        uint64_t off = 0;
        if ((s = pend_reserve(c, L, var, m, &off))) return s;
        uint32_t* codes = (uint32_t*)c->part_codes.p + off * G;
        uint16_t* inval = (uint16_t*)c->part_inval.p + off * G;
        if (var) {
            HIPCHK(c, launch_encode_reads_var(base, seq_off + done, seq_end + done, m, (int)L, (int)c->k, codes, inval,
                                              (uint16_t*)c->part_rlen.p + off, c->stats, c->stream));
        } else {
            CountLaunch l;
            l.base = base;
            l.seq_off = seq_off;
            l.read0 = done;
            l.n_reads = m;
            l.L = (int)L;
            l.k = (int)c->k;
            HIPCHK(c, launch_encode_reads(l, codes, inval, c->stream, c->stats));
            if (c->pend_sparse)  // rows of a one-pass batch carry their length
                HIPCHK(c, hipMemsetD16Async((hipDeviceptr_t)((uint16_t*)c->part_rlen.p + off), (unsigned short)L, m,
                                            c->stream));
        }
        c->pend_reads += m;
        done += m;
    }
    return KC_OK;
}

// The engine count_reads takes for L reads (same order of tests): the skm and
// key-prefix engines read 2-bit codes, the table engine the text
static bool engine_reads_codes(const kc_ctx* c, int64_t L) {
    if (c->skm && !c->skm_hc && skm_geometry((int)L, (int)c->k).ok) return true;
    return c->part && part_geometry((int)L, (int)c->k, 1).lds_scatter <= kMaxLds;
}

// K1 for one record-aligned FASTQ block in device memory (GPU FASTQ decode,
// replacing FASTQFileReader::readData, FASTQFileReader.cpp:49-89): newline
// counts per 16 KiB chunk -> each chunk's first line index -> one of
//   fused   : index + checks + 2-bit encode in one read of the text, straight
//             into the pending batch (fq_encode_k; fq_encode_k<true> for
//             variable-length reads), when the block fits the pending room;
//   two-pass: sequence offsets (fq_emit_k) + length check (fq_validate_k),
//             then encode per batch (kernel E) — blocks larger than a batch,
//             and the table engine, which counts the text itself.
// The whole block is checked before any of its reads is pending or counted: a
// malformed block changes nothing and returns KC_ERR_FORMAT. With count =
// false only the checks run (kc_check_fastq).
static std::string fq_errors(uint64_t e, bool var) {
    std::string why;
    if (e & ERR_FQ_NOT_AT) why += " record-does-not-start-with-@";
    if (e & ERR_FQ_NO_PLUS) why += " no-+-line-after-sequence";
    if (e & ERR_FQ_SEQ_LEN) why += var ? " sequence-longer-than-L" : " sequence-length-differs-from-L";
    if (e & ERR_FQ_TOO_MANY) why += " index-overflow";
    if (e & ERR_FQ_NO_FINAL_NL) why += " block-does-not-end-with-newline";
    return why;
}

static kc_status ingest_fastq(kc_ctx* c, const uint8_t* base, uint64_t n, int64_t L, bool var, bool count,
                              uint64_t* n_rec_out, bool two_pass = false, bool no_spec = false) {
    kc_status s;
    uint64_t nch = fq_chunks(base, n);
    if ((s = ensure(c, c->fq_counts, nch * 8 + 16)) || (s = ensure(c, c->fq_base, nch * 8)) ||
        (s = ensure(c, c->fq_tmp, scan_tmp_elems(nch) * 8)))
        return s;
    if ((s = sync_stats(c))) return s;
    uint64_t snap[ST_N];
    memcpy(snap, c->stats_h, sizeof(snap));
    auto restore = [&]() -> kc_status {
        // the counters the index / encode kernels touched (errors, variable-length hole flag and windows)
        snap[ST_ERR] = 0;
        HIPCHK(c, hipMemcpyAsync(c->stats, snap, sizeof(snap), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        memcpy(c->stats_h, snap, sizeof(snap));
        return KC_OK;
    };
    // One-pass index (fixed L, codes engines): the text is read once; every
    // chunk guesses its line phase and writes its records to rows of its own,
    // then the guesses are checked against the scanned newline counts. A miss
    // or any error: the block is indexed again by the path below, which also
    // gives format errors their verdict.
    // Only where the super-k-mer engine's F3 front end will read the rows (it
    // skips an empty row for free): the key-prefix front end walks them
    // (cfg5, k = 55: P1 + P2 +1.5 ms against 0.7 ms saved in the index,
    // same-box A/B), as do F2 and the W >= 2 front ends
    // (the same conditions as F3's own choice: skm engine not
    // handed over to the key-prefix engine, F3's geometry and LDS budget)
    const bool f3_rows = c->skm && !c->skm_hc && c->W == 1 && c->k >= 19 && c->k <= 32 &&
                         skm_f3_applies((int)L, (int)c->k);
    const bool spec = count && !var && !two_pass && !no_spec && f3_rows && engine_reads_codes(c, L) &&
                      fq_spec_ok((int)L) && !test_hook("KC_NO_FQ_ENCODE") && !test_hook("KC_NO_FQ_SPEC");
    const uint64_t spec_rows = spec ? nch * fq_spec_rows_per_chunk((int)L) : 0;
    if (spec && spec_rows <= pend_room(c, L)) {
        uint64_t off = 0;
        if ((s = pend_reserve(c, L, false, spec_rows, &off, true)) || (s = ensure(c, c->fq_phase, nch + 16)))
            return s;
        const uint64_t G = (uint64_t)groups_per_read((int)L);
        HIPCHK(c, hipEventRecord(c->ev0, c->stream));
        HIPCHK(c, hipMemsetAsync(c->stats + ST_ERR, 0, 8, c->stream));
        HIPCHK(c, launch_fq_encode_spec(base, n, (int)L, (uint32_t*)c->part_codes.p + off * G,
                                        (uint16_t*)c->part_inval.p + off * G, (uint16_t*)c->part_rlen.p + off,
                                        (uint64_t*)c->fq_counts.p, (uint8_t*)c->fq_phase.p, c->stats, c->stream));
        HIPCHK(c, launch_scan_u64((uint64_t*)c->fq_counts.p, (uint64_t*)c->fq_base.p, nch, (uint64_t*)c->fq_tmp.p,
                                  c->stream));
        HIPCHK(c, launch_fq_spec_verify((const uint64_t*)c->fq_base.p, (const uint8_t*)c->fq_phase.p, nch, c->stats,
                                        c->stream));
        // [nch]: the line total; [nch + 1]: the rows per chunk the kernel used
        uint64_t* total = (uint64_t*)c->fq_counts.p + nch;
        HIPCHK(c, launch_sum_last((const uint64_t*)c->fq_base.p, (const uint64_t*)c->fq_counts.p, nch, total, c->stream));
        uint64_t lr[2] = {0, 0};
        HIPCHK(c, hipMemcpyAsync(lr, total, 16, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipEventRecord(c->ev1, c->stream));
        if ((s = sync_stats(c))) return s;
        float t = 0.f;
        HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
        c->st.decode_ms += t;
        const uint64_t lines = lr[0];
        if (c->stats_h[ST_ERR] == 0 && lines % 4 == 0 && lines > 0 && lr[1] >= 1 &&
            lr[1] <= fq_spec_rows_per_chunk((int)L)) {
            const uint64_t n_rec = lines / 4;
            if (n_rec_out) *n_rec_out = n_rec;
            // rows the kernel used (<= the reserved spec_rows). The pending
            // batch counts rows, empty ones included (~4% at cfg2's headers, up
            // to ~15% for short headers): batch sizing, the record pool's
            // reservation and the sketch's sampling rate treat every row as a
            // read, so they err on the safe side (more room reserved, a few
            // more samples); st.reads and st.windows count the real records
            c->pend_reads += nch * lr[1];
            c->pend_sparse = true;
            c->st.reads += n_rec;
            c->st.windows += n_rec * (uint64_t)(L - c->k + 1);
            return KC_OK;
        }
        if (getenv("KC_DEBUG"))
            fprintf(stderr, "kc: one-pass FASTQ index missed (errors %#llx, %llu lines): two-kernel index\n",
                    (unsigned long long)c->stats_h[ST_ERR], (unsigned long long)lines);
        if ((s = restore())) return s;
        return ingest_fastq(c, base, n, L, var, count, n_rec_out, false, true);
    }
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, hipMemsetAsync(c->stats + ST_ERR, 0, 8, c->stream));
    HIPCHK(c, launch_fq_count(base, n, (uint64_t*)c->fq_counts.p, c->stream));
    HIPCHK(c, launch_scan_u64((uint64_t*)c->fq_counts.p, (uint64_t*)c->fq_base.p, nch, (uint64_t*)c->fq_tmp.p,
                              c->stream));
    // the line count (last chunk's base + count, summed on the device: one readback)
    uint64_t* total = (uint64_t*)c->fq_counts.p + nch;
    HIPCHK(c, launch_sum_last((const uint64_t*)c->fq_base.p, (const uint64_t*)c->fq_counts.p, nch, total, c->stream));
    uint64_t lines = 0;
    HIPCHK(c, hipMemcpyAsync(&lines, total, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (lines % 4 != 0)
        return fail(c, KC_ERR_FORMAT, "FASTQ block has %llu lines, not a multiple of 4", (unsigned long long)lines);
    const uint64_t n_rec = lines / 4;
    const uint64_t G = (uint64_t)groups_per_read((int)L);
    const bool codes = engine_reads_codes(c, L);
    if (var && (!c->part || !codes))
        return fail(c, KC_ERR_ARG, "variable-length reads need an engine that reads encoded reads (L = %lld)",
                    (long long)L);
    // where the block's reads go: the pending batch when they fit it (after
    // counting a pending batch of another kind or too full to take them)
    uint64_t off = 0;
    // (count = false, kc_check_fastq: the two-pass index checks the block and
    // nothing is reserved, encoded or flushed: a validation has no side effects)
    const bool into_pend = count && codes && n_rec > 0 && n_rec <= pend_room(c, L, var);
    if (into_pend && (s = pend_reserve(c, L, var, n_rec, &off))) return s;
    const bool no_fuse = test_hook("KC_NO_FQ_ENCODE") != nullptr;  // path selector (tests): same bytes either way
    const bool fused = into_pend && !var && !no_fuse;                               // fq_encode_k
    const bool whole_var = into_pend && var;                                         // the block encoded whole
    const bool fused_var = whole_var && !two_pass && !no_fuse && fq_encode_var_ok((int)L);  // fq_encode_k<true>
    if (fused) {
        HIPCHK(c, launch_fq_encode(base, n, (uint64_t*)c->fq_base.p, n_rec, (int)L,
                                   (uint32_t*)c->part_codes.p + off * G, (uint16_t*)c->part_inval.p + off * G,
                                   c->stats, c->stream));
    } else if (fused_var) {
        HIPCHK(c, launch_fq_encode_var(base, n, (uint64_t*)c->fq_base.p, n_rec, (int)L, (int)c->k,
                                       (uint32_t*)c->part_codes.p + off * G, (uint16_t*)c->part_inval.p + off * G,
                                       (uint16_t*)c->part_rlen.p + off, c->stats, c->stream));
    } else {
        if ((s = ensure(c, c->seq_off, n_rec * 8 + 8)) || (s = ensure(c, c->seq_end, n_rec * 8 + 8))) return s;
        HIPCHK(c, launch_fq_emit(base, n, (uint64_t*)c->fq_base.p, (uint64_t*)c->seq_off.p, (uint64_t*)c->seq_end.p,
                                 n_rec, c->stats, c->stream));
        HIPCHK(c, launch_fq_validate((uint64_t*)c->seq_off.p, (uint64_t*)c->seq_end.p, n_rec, (int)L, c->stats,
                                     c->stream, var));
        if (whole_var)
            HIPCHK(c, launch_encode_reads_var(base, (const uint64_t*)c->seq_off.p, (const uint64_t*)c->seq_end.p,
                                              n_rec, (int)L, (int)c->k, (uint32_t*)c->part_codes.p + off * G,
                                              (uint16_t*)c->part_inval.p + off * G, (uint16_t*)c->part_rlen.p + off,
                                              c->stats, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    if ((s = sync_stats(c))) return s;
    float t = 0.f;
    HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
    c->st.decode_ms += t;
    const uint64_t e = c->stats_h[ST_ERR];
    if (fused_var && (e & ERR_FQ_LIST)) {
        // a half held more records than the fused list: the two-pass index
        if ((s = restore())) return s;
        return ingest_fastq(c, base, n, L, var, count, n_rec_out, true, no_spec);
    }
    if (e) {
        const std::string why = fq_errors(e, var);
        if ((s = restore())) return s;
        return fail(c, KC_ERR_FORMAT, "FASTQ block is not 4-line records with %s%lld-base reads:%s",
                    var ? "at most " : "", (long long)L, why.c_str());
    }
    if (n_rec_out) *n_rec_out = n_rec;
    if (!count) return var ? restore() : KC_OK;  // (the encoded reads past pend_reads are dropped)
    const uint64_t vwin0 = snap[ST_VWIN];
    c->st.reads += n_rec;
    if (fused || whole_var) {
        if (fused && c->pend_sparse)  // rows of a one-pass batch carry their length
            HIPCHK(c, hipMemsetD16Async((hipDeviceptr_t)((uint16_t*)c->part_rlen.p + off), (unsigned short)L, n_rec,
                                        c->stream));
        c->pend_reads += n_rec;
    } else if (codes) {
        if ((s = pend_add_reads(c, base, (const uint64_t*)c->seq_off.p, (const uint64_t*)c->seq_end.p, n_rec, L, var)))
            return s;
    } else {
        // the table engine reads the text: counted now
        if ((s = pend_flush(c))) return s;
        if ((s = count_reads(c, base, (const uint64_t*)c->seq_off.p, n_rec, L))) return s;
    }
    if (var) {
        if ((s = sync_stats(c))) return s;
        c->st.windows += c->stats_h[ST_VWIN] - vwin0;  // the reads' own windows, not the padded slots'
    } else {
        c->st.windows += n_rec * (uint64_t)(L - c->k + 1);
    }
    return KC_OK;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------

extern "C" {

int32_t kc_abi_version(void) { return KC_ABI_VERSION; }

int32_t kc_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* kc_strerror(kc_status s) {
    switch (s) {
    case KC_OK: return "ok";
    case KC_ERR_ARG: return "invalid argument";
    case KC_ERR_HIP: return "HIP runtime error";
    case KC_ERR_NOMEM: return "out of memory";
    case KC_ERR_FORMAT: return "malformed FASTQ block";
    case KC_ERR_IO: return "I/O error";
    case KC_ERR_STATE: return "invalid call for the context state";
    case KC_ERR_NODEVICE: return "no HIP device";
    case KC_ERR_INTERNAL: return "internal error";
    }
    return "unknown status";
}

const char* kc_last_error(const kc_ctx* c) { return c ? c->err.c_str() : ""; }

kc_status kc_create(kc_ctx** out, const kc_config* cfg) {
    if (!out || !cfg) return KC_ERR_ARG;
    *out = nullptr;
    if (cfg->kmer_length < 1 || cfg->kmer_length > KC_MAX_K) return KC_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return KC_ERR_NODEVICE;
    if (cfg->device < 0 || cfg->device >= ndev) return KC_ERR_NODEVICE;
    kc_ctx* c = new kc_ctx();
    c->cfg = *cfg;
    c->temp_dir = (cfg->temp_dir && cfg->temp_dir[0]) ? cfg->temp_dir : "";
    c->cfg.temp_dir = nullptr;
    c->k = cfg->kmer_length;
    c->W = (int)((c->k + 31) / 32);
    c->rs = 8 * c->W + 4;
    c->id = g_ctx_seq.fetch_add(1);
    memset(&c->st, 0, sizeof(c->st));
    kc_status s = KC_OK;
    auto bail = [&](kc_status e) {
        kc_destroy(c);
        return e;
    };
    if (hipSetDevice(cfg->device) != hipSuccess) return bail(KC_ERR_NODEVICE);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bail(KC_ERR_HIP);
    if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev2) != hipSuccess || hipEventCreate(&c->evf[0]) != hipSuccess ||
        hipEventCreate(&c->evf[1]) != hipSuccess)
        return bail(KC_ERR_HIP);
    uint64_t M = cfg->gpu_memory_limit ? cfg->gpu_memory_limit : 100000000ull;
    if (M < (1u << 20)) M = 1u << 20;
    if ((cfg->flags & KC_FLAG_VARLEN) && (cfg->flags & KC_FLAG_ENGINE_TABLE)) {
        delete c;
        return KC_ERR_ARG;  // the table engine reads the text, not encoded reads
    }
    c->part = (cfg->flags & KC_FLAG_ENGINE_TABLE) == 0;
    c->skm = c->part && (cfg->flags & KC_FLAG_ENGINE_PREFIX) == 0;
    c->skm_force = (cfg->flags & KC_FLAG_ENGINE_SKM) != 0;
    size_t slot_bytes = 8 * (size_t)slot_words(c->W);
    size_t spill_bytes, tbytes;
    if (c->part) {
        // partition engine: two key buffers take the working set; the global
        // table and spill buffer only catch LDS-table overflow
        spill_bytes = M / 64;
        tbytes = cfg->table_bytes ? cfg->table_bytes : M / 16;
        uint64_t rest = M - M / 64 - M / 16;
        c->key_cap = rest / (16 * (uint64_t)c->W + 1);  // two key buffers + the P3 digit byte
        if (c->key_cap < 65536) c->key_cap = 65536;
    } else {
        spill_bytes = M / 16;
        tbytes = cfg->table_bytes ? cfg->table_bytes : (M - 4 * spill_bytes);
    }
    c->spill_cap = spill_bytes / (8 * c->W);
    if (c->spill_cap < 4096) c->spill_cap = 4096;
    c->cap = tbytes / slot_bytes;
    if (c->cap < 1024) c->cap = 1024;
    c->table_bytes = c->cap * slot_bytes;
    if (hipMalloc((void**)&c->table, c->table_bytes) != hipSuccess) return bail(KC_ERR_NOMEM);
    if (hipMalloc((void**)&c->spill, (size_t)c->spill_cap * 8 * c->W) != hipSuccess) return bail(KC_ERR_NOMEM);
    if (hipMalloc((void**)&c->stats, ST_N * 8) != hipSuccess) return bail(KC_ERR_NOMEM);
    if (hipHostMalloc((void**)&c->stats_h, ST_N * 8, 0) != hipSuccess) return bail(KC_ERR_NOMEM);
    if (c->part) {
        if (hipMalloc((void**)&c->keys_a, (size_t)c->key_cap * 8 * c->W) != hipSuccess) return bail(KC_ERR_NOMEM);
        if (hipMalloc((void**)&c->keys_b, (size_t)c->key_cap * 8 * c->W) != hipSuccess) return bail(KC_ERR_NOMEM);
        // key_cap digit bytes for the partition engine; the skm engine's two digit
        // arrays (2 x pool_cap, pool_cap = W key_cap / (W + 1)) with the second one
        // 16-byte aligned
        c->digs_bytes = c->key_cap;
        const uint64_t pool_max = (uint64_t)c->W * c->key_cap / (c->W + 1);
        if (((pool_max + 15) & ~15ull) + pool_max > c->digs_bytes) c->digs_bytes = ((pool_max + 15) & ~15ull) + pool_max;
        if (hipMalloc((void**)&c->digs, (size_t)c->digs_bytes + 16) != hipSuccess) return bail(KC_ERR_NOMEM);
        if (hipMalloc((void**)&c->rec_cursor, 8) != hipSuccess) return bail(KC_ERR_NOMEM);
        if (hipMalloc((void**)&c->pool_cursor, 8) != hipSuccess) return bail(KC_ERR_NOMEM);
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, cfg->device) == hipSuccess && prop.multiProcessorCount > 0)
            c->n_cu = prop.multiProcessorCount;
    }
    size_t mfree = 0, mtotal = 0;
    if (hipMemGetInfo(&mfree, &mtotal) == hipSuccess) c->dev_total = mtotal;
    s = kc_reset(c);
    if (s) return bail(s);
    *out = c;
    return KC_OK;
}

void kc_destroy(kc_ctx* c) {
    if (!c) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    delete c->ring;  // waits for its DMAs
    delete c->pool;
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    for (char* b : c->file_bufs) (void)hipHostFree(b);
    for (int i = 0; i < 2; i++) {
        if (c->acc_buf[i]) (void)hipHostFree(c->acc_buf[i]);
        if (c->acc_ev[i]) (void)hipEventDestroy(c->acc_ev[i]);
    }
    for (auto& b : c->file_stage) release(b);
    for (auto& e : c->file_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->stage_free)
        if (e) (void)hipEventDestroy(e);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    release_dev_runs(c, true);
    for (auto& r : c->runs)
        if (!r.path.empty()) unlink(r.path.c_str());
    DevBuf* bufs[] = {&c->in_stage, &c->fq_counts, &c->fq_base, &c->fq_tmp, &c->seq_off, &c->seq_end,
                      &c->spill_keys2, &c->rle_flags, &c->rle_pos, &c->rle_head, &c->rle_tmp, &c->run_keys,
                      &c->run_cnts, &c->run_packed, &c->fin_keys[0], &c->fin_keys[1], &c->fin_cnts[0],
                      &c->fin_cnts[1], &c->fin_hist, &c->fin_packed, &c->fin_misc, &c->merge_tmp};
    for (DevBuf* b : bufs) release(*b);
    if (c->table) (void)hipFree(c->table);
    if (c->spill) (void)hipFree(c->spill);
    if (c->keys_a) (void)hipFree(c->keys_a);
    if (c->keys_b) (void)hipFree(c->keys_b);
    if (c->digs) (void)hipFree(c->digs);
    if (c->rec_keys) (void)hipFree(c->rec_keys);
    if (c->rec_dig) (void)hipFree(c->rec_dig);
    if (c->rec_cnts) (void)hipFree(c->rec_cnts);
    if (c->rec_cursor) (void)hipFree(c->rec_cursor);
    if (c->pool_cursor) (void)hipFree(c->pool_cursor);
    release(c->part_hist);
    release(c->part_ghist);
    release(c->part_base2);
    release(c->p3b_buf);
    release(c->run_flags);
    release(c->sub_starts);
    release(c->part_codes);
    release(c->part_inval);
    release(c->part_rlen);
    DevBuf* dbufs[] = {&c->desc_key, &c->desc_start, &c->desc_len, &c->desc_k2, &c->desc_v, &c->desc_v2,
                       &c->desc_lens, &c->desc_offs, &c->desc_fb};
    for (DevBuf* b : dbufs) release(*b);
    release(c->part_base);
    release(c->part_tmp);
    release(c->part_starts);
    release(c->part_sort_hist);
    if (c->stats) (void)hipFree(c->stats);
    if (c->stats_h) (void)hipHostFree(c->stats_h);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    for (hipEvent_t e : c->evf)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

kc_status kc_reset(kc_ctx* c) {
    if (!c) return KC_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    // the global table is cleared only when a slot was claimed since the last
    // clear (the partition engine's table is a rarely used fallback: clearing
    // 1/16 of gpuMemoryLimit per reset would cost milliseconds per count)
    kc_status s0 = sync_stats(c);
    if (s0) return s0;
    if (c->table_dirty || c->stats_h[ST_CLAIMED] > 0) {
        HIPCHK(c, hipMemsetAsync(c->table, 0, c->table_bytes, c->stream));
        c->table_dirty = false;
    }
    HIPCHK(c, hipMemsetAsync(c->stats, 0, ST_N * 8, c->stream));
    if (c->rec_cursor) HIPCHK(c, hipMemsetAsync(c->rec_cursor, 0, 8, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    memset(c->stats_h, 0, ST_N * 8);
    c->rec_n = 0;
    c->batches = 0;
    for (double& x : c->part_ms) x = 0;
    c->presplit_ms = 0;
    c->presplit_batches = 0;
    c->sorted_run_batches = 0;
    c->key_passes = 0;
    c->dedup_ms = 0;
    c->finish_group_ms = 0;
    c->dedup_records = 0;
    c->part_keys = 0;
    c->p5_launches = 0;
    c->skm_used = false;
    c->skm_checked = false;
    c->skm_big_off = false;
    c->skm_hc = false;
    c->hc_hint = false;
    c->engines_used = 0;
    for (auto& r : c->runs)
        if (!r.path.empty()) unlink(r.path.c_str());
    c->runs.clear();
    c->spilled_flushed = 0;
    release_dev_runs(c, false);
    c->runs_cut = 0;
    c->batches_cut = 0;
    c->pend_reads = 0;
    c->pend_L = 0;
    c->pend_var = false;
    c->pend_sparse = false;
    c->acc_n = 0;  // (a DMA still reading a buffer is waited for before it is refilled)
    c->ckpt = false;
    c->finished = false;
    c->n_records = 0;
    memset(&c->st, 0, sizeof(c->st));
    c->st.table_capacity = c->cap;
    return KC_OK;
}

// Host staging (pinned ring + copy pool), created on first use.
static kc_status stage_init(kc_ctx* c) {
    if (!c->pool) {
        // host copy threads: the CPUs this process may run on, at most 16 (the
        // GPU box's cgroup quota; its affinity mask shows every core)
        cpu_set_t cs;
        int n = 8;
        if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = CPU_COUNT(&cs);
        c->pool = new kc::Pool(std::max(2, std::min(16, n)));
    }
    if (!c->ring) {
        c->ring = new kc::PinnedRing();
        HIPCHK(c, c->ring->init((size_t)64 << 20, 4));
    }
    return KC_OK;
}

// Reference-exact chunk in device memory: floor(size / L) reads at stride L
// (GPUHandler.cu:13-15), encoded into the pending batch (codes engines) or
// counted from the text (table engine).
static kc_status chunk_device(kc_ctx* c, const uint8_t* d, int64_t size, int64_t L, bool add_stats = true) {
    if (c->finished) return fail(c, KC_ERR_STATE, "kc_finish was called; kc_reset first");
    const uint64_t n = (uint64_t)(size / L);
    if (n == 0) return KC_OK;
    kc_status s;
    if (engine_reads_codes(c, L)) {
        if ((s = pend_add_reads(c, d, nullptr, nullptr, n, L, false))) return s;
    } else {
        if ((s = pend_flush(c))) return s;
        if ((s = count_reads(c, d, nullptr, n, L))) return s;
    }
    if (add_stats) {
        c->st.reads += n;
        c->st.windows += n * (uint64_t)(L - c->k + 1);
    }
    return KC_OK;
}

kc_status kc_count_chunk_device(kc_ctx* c, const void* d_chunk, int64_t size, int64_t L) {
    if (!c || (!d_chunk && size > 0) || size < 0) return KC_ERR_ARG;
    kc_status s = check_line(c, L);
    if (s) return s;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if ((s = chunk_acc_flush(c))) return s;
    if ((s = chunk_device(c, (const uint8_t*)d_chunk, size, L))) return s;
    HIPCHK(c, hipStreamSynchronize(c->stream));  // the caller's buffer was read by the encoder
    return KC_OK;
}

static kc_status copy_stream_init(kc_ctx* c) {
    if (c->copy_stream) return KC_OK;
    HIPCHK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (auto& e : c->file_ev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : c->stage_free) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return KC_OK;
}

// One staged upload + encode of host bytes (whole reads of length L): through
// the pinned ring (pageable source) or straight from a pinned buffer, into one
// of two staging buffers on the copy stream; the encode waits for that upload
// on the ctx stream, so the next upload overlaps this encode.
static kc_status chunk_upload_count(kc_ctx* c, const char* src, size_t bytes, int64_t L, bool pinned_src,
                                    hipEvent_t src_done, bool add_stats) {
    kc_status s;
    const int slot = c->chunk_slot;
    c->chunk_slot ^= 1;
    DevBuf& st = c->file_stage[slot];
    if (st.bytes < bytes + 64) {
        // growing: nothing may still read or write the old buffer
        HIPCHK(c, hipStreamSynchronize(c->copy_stream));
        if ((s = ensure(c, st, bytes + 64))) return s;
    }
    HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->stage_free[slot], 0));
    if (pinned_src) {
        HIPCHK(c, hipMemcpyAsync(st.p, src, bytes, hipMemcpyHostToDevice, c->copy_stream));
        if (src_done) HIPCHK(c, hipEventRecord(src_done, c->copy_stream));
    } else {
        HIPCHK(c, c->ring->upload(st.p, src, bytes, c->copy_stream, c->pool));
    }
    HIPCHK(c, hipEventRecord(c->file_ev[slot], c->copy_stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->file_ev[slot], 0));
    if ((s = chunk_device(c, (const uint8_t*)st.p, (int64_t)bytes, L, add_stats))) return s;
    HIPCHK(c, hipEventRecord(c->stage_free[slot], c->stream));
    return KC_OK;
}

static const size_t kAccBytes = (size_t)64 << 20;

// Uploads and counts the accumulated chunk reads (kc_count_chunk), if any.
static kc_status chunk_acc_flush(kc_ctx* c) {
    if (!c->acc_n) return KC_OK;
    const size_t bytes = c->acc_n;
    const int i = c->acc_i;
    c->acc_n = 0;  // first: counting may flush the pending batch, which comes back here
    c->acc_i ^= 1;
    c->acc_busy[i] = true;
    return chunk_upload_count(c, c->acc_buf[i], bytes, c->acc_L, true, c->acc_ev[i], false);
}

// Host chunk (the reference's readData output, KMerCounter.cpp:193-212: ~7.8
// MB at gpuMemoryLimit=1e8): its whole reads are copied into the pinned
// accumulation buffer (the call returns once the caller's bytes are copied);
// a full buffer (64 MB, about 8 such chunks) is uploaded and encoded while the
// next one fills, so per chunk the cost is the host copy and no device call.
// A chunk larger than half the buffer goes through the pinned ring directly.
kc_status kc_count_chunk(kc_ctx* c, const char* chunk, int64_t size, int64_t L) {
    if (!c || (!chunk && size > 0) || size < 0) return KC_ERR_ARG;
    kc_status s = check_line(c, L);
    if (s) return s;
    const uint64_t n = (uint64_t)(size / L);
    if (n == 0) return KC_OK;
    if (c->finished) return fail(c, KC_ERR_STATE, "kc_finish was called; kc_reset first");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if ((s = stage_init(c)) || (s = copy_stream_init(c))) return s;
    const size_t bytes = (size_t)(n * (uint64_t)L);
    const bool tr = kc::trace_on();
    double t0 = tr ? kc::now_s() : 0;
    if (tr) c->acc_t[3] += 1;
    if (c->acc_n && (c->acc_L != L || c->acc_n + bytes > kAccBytes))
        if ((s = chunk_acc_flush(c))) return s;
    if (tr) {
        const double t = kc::now_s();
        c->acc_t[2] += t - t0;
        t0 = t;
    }
    if (bytes > kAccBytes / 2) return chunk_upload_count(c, chunk, bytes, L, false, nullptr, true);
    const int i = c->acc_i;
    if (!c->acc_buf[i]) {
        HIPCHK(c, hipHostMalloc((void**)&c->acc_buf[i], kAccBytes, hipHostMallocDefault));
        HIPCHK(c, hipEventCreateWithFlags(&c->acc_ev[i], hipEventDisableTiming));
    }
    if (c->acc_n == 0) {
        if (c->acc_busy[i]) {  // its previous upload must be done before it is refilled
            HIPCHK(c, hipEventSynchronize(c->acc_ev[i]));
            c->acc_busy[i] = false;
        }
        c->acc_L = L;
    }
    if (tr) {
        const double t = kc::now_s();
        c->acc_t[1] += t - t0;
        t0 = t;
    }
    kc::par_memcpy(c->pool, c->acc_buf[i] + c->acc_n, chunk, bytes);
    if (tr) c->acc_t[0] += kc::now_s() - t0;
    c->acc_n += bytes;
    c->st.reads += n;
    c->st.windows += n * (uint64_t)(L - c->k + 1);
    return KC_OK;
}

static kc_status fastq_device(kc_ctx* c, const void* d_fastq, uint64_t n, int64_t L, uint64_t* n_reads,
                              bool count) {
    if (!c || (!d_fastq && n > 0)) return KC_ERR_ARG;
    if (n_reads) *n_reads = 0;
    if (n == 0) return KC_OK;
    if (count && c->finished) return fail(c, KC_ERR_STATE, "kc_finish was called; kc_reset first");
    if (L == 0) L = c->cfg.line_length;
    kc_status s = check_line(c, L);
    if (s) return s;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if (count && (s = chunk_acc_flush(c))) return s;
    return ingest_fastq(c, (const uint8_t*)d_fastq, n, L, (c->cfg.flags & KC_FLAG_VARLEN) != 0, count, n_reads);
}

// Host FASTQ block: uploaded through the pinned ring (pageable) or directly
// (pinned), then decoded on the GPU (ingest_fastq, which waits for the
// checks: a malformed block is reported by this call).
static kc_status fastq_host(kc_ctx* c, const char* fastq, uint64_t n, int64_t L, uint64_t* n_reads, bool count) {
    if (!c || (!fastq && n > 0)) return KC_ERR_ARG;
    if (n_reads) *n_reads = 0;
    if (n == 0) return KC_OK;
    kc_status s;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if ((s = stage_init(c))) return s;
    if ((s = ensure(c, c->in_stage, (size_t)n + 64))) return s;
    HIPCHK(c, c->ring->upload(c->in_stage.p, fastq, n, c->stream, c->pool));
    return fastq_device(c, c->in_stage.p, n, L, n_reads, count);
}

kc_status kc_count_fastq_device(kc_ctx* c, const void* d_fastq, uint64_t n, int64_t L, uint64_t* n_reads) {
    return fastq_device(c, d_fastq, n, L, n_reads, true);
}

kc_status kc_count_fastq(kc_ctx* c, const char* fastq, uint64_t n, int64_t L, uint64_t* n_reads) {
    return fastq_host(c, fastq, n, L, n_reads, true);
}

kc_status kc_check_fastq(kc_ctx* c, const char* fastq, uint64_t n, int64_t L, uint64_t* n_reads) {
    return fastq_host(c, fastq, n, L, n_reads, false);
}

// ---- file input (InputFileHandler / FASTQFileReader + the Start loop) ----

static const size_t kFileBlock = (size_t)256 << 20;

// Block size of the file reader; KC_FILE_BLOCK (bytes) is a path selector for
// tests (many blocks from small files: cut search, carries; same counts).
static size_t file_block_bytes() {
    if (const char* e = test_hook("KC_FILE_BLOCK")) {
        const long long v = atoll(e);
        if (v >= 4096) return (size_t)v;
    }
    return kFileBlock;
}

// Uploads a block of the file reader (pinned) into staging buffer `slot` on
// the ctx's copy stream; the decode waits for it through file_ev[slot].
static kc_status file_upload(kc_ctx* c, int slot, const char* p, size_t n) {
    kc_status s;
    if ((s = copy_stream_init(c))) return s;
    if (c->file_stage[slot].bytes < n + 64) {
        HIPCHK(c, hipStreamSynchronize(c->copy_stream));
        if ((s = ensure(c, c->file_stage[slot], n + 64))) return s;
    }
    HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->stage_free[slot], 0));  // a chunk encode may still read it
    HIPCHK(c, hipMemcpyAsync(c->file_stage[slot].p, p, n, hipMemcpyHostToDevice, c->copy_stream));
    HIPCHK(c, hipEventRecord(c->file_ev[slot], c->copy_stream));
    return KC_OK;
}

// The GPU decode of an uploaded block (waits for its checks, hence for the
// upload: the reader may refill the host block when this returns). Kernels
// queued by the decode may still read the staging buffer (an encode of reads
// appended to the pending batch is not waited for), so the next upload into
// this slot waits for stage_free[slot], recorded after them.
static kc_status file_decode(kc_ctx* c, int slot, size_t n, int64_t L, bool count, uint64_t* got) {
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->file_ev[slot], 0));
    kc_status s = fastq_device(c, c->file_stage[slot].p, n, L, got, count);
    HIPCHK(c, hipEventRecord(c->stage_free[slot], c->stream));
    return s;
}

// Streams the file's blocks to the contexts (each block to whichever context
// is free: counting is order-independent). On the first failing block every
// context stops; *failed names the context that reported it.
static kc_status file_blocks(kc_ctx* const* ctxs, uint32_t n_ctx, const char* path, int64_t L, bool count,
                             uint64_t* reads, kc_ctx** failed) {
    // the reader's pinned buffers live in ctxs[0] (2 n_ctx + 2 of them: two per
    // context in flight, one filling, one holding the carried tail)
    kc_ctx* c0 = ctxs[0];
    const size_t block = file_block_bytes();
    const size_t want = block + kc::FastqFileReader::carry_bytes();
    if (c0->file_buf_bytes != want) {
        for (char* b : c0->file_bufs) (void)hipHostFree(b);
        c0->file_bufs.clear();
        c0->file_buf_bytes = want;
    }
    HIPCHK(c0, hipSetDevice(c0->cfg.device));
    while (c0->file_bufs.size() < 2 * (size_t)n_ctx + 2) {
        char* b = nullptr;
        HIPCHK(c0, hipHostMalloc((void**)&b, want, 0));
        c0->file_bufs.push_back(b);
    }
    std::vector<char*> bufs(c0->file_bufs.begin(), c0->file_bufs.begin() + 2 * n_ctx + 2);
    kc::FastqFileReader rd(block, bufs, 8);
    std::string err;
    *failed = ctxs[0];
    if (!rd.open(path, &err)) return fail(ctxs[0], KC_ERR_IO, "%s", err.c_str());
    std::atomic<bool> stop(false);
    std::vector<kc_status> st(n_ctx, KC_OK);
    std::vector<uint64_t> nr(n_ctx, 0);
    // per context: block i + 1 is uploaded (copy stream) while block i is
    // decoded (ctx stream)
    auto work = [&](uint32_t g) {
        kc_ctx* c = ctxs[g];
        if (hipSetDevice(c->cfg.device) != hipSuccess) {
            st[g] = fail(c, KC_ERR_HIP, "hipSetDevice(%d)", c->cfg.device);
            stop = true;
            return;
        }
        kc::FastqFileReader::Block cur, nxt;
        bool have = !stop && rd.next(&cur);
        int slot = 0;
        kc_status s = have ? file_upload(c, slot, cur.p, cur.n) : KC_OK;
        while (have && !s) {
            const bool have_nxt = !stop && rd.next(&nxt);
            if (have_nxt && (s = file_upload(c, slot ^ 1, nxt.p, nxt.n))) {
                rd.release(nxt);
                break;
            }
            uint64_t got = 0;
            const double t0 = kc::trace_on() ? kc::now_s() : 0;
            s = file_decode(c, slot, cur.n, L, count, &got);
            if (kc::trace_on()) kc::trace("ctx %u block %llu: %zu bytes, decode (+ upload wait) %.3f ms", g,
                                          (unsigned long long)cur.index, cur.n, (kc::now_s() - t0) * 1e3);
            rd.release(cur);
            nr[g] += got;
            if (s) {
                if (have_nxt) {
                    (void)hipStreamSynchronize(c->copy_stream);
                    rd.release(nxt);
                }
                break;
            }
            cur = nxt;
            have = have_nxt;
            slot ^= 1;
        }
        if (s) {
            st[g] = s;
            stop = true;
        }
    };
    if (n_ctx == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (uint32_t g = 0; g < n_ctx; g++) th.emplace_back(work, g);
        for (auto& t : th) t.join();
    }
    for (uint32_t g = 0; g < n_ctx; g++)
        if (st[g]) {
            *failed = ctxs[g];
            return st[g];
        }
    err = rd.error();
    if (!err.empty()) return fail(ctxs[0], KC_ERR_IO, "%s: %s", path, err.c_str());
    for (uint32_t g = 0; g < n_ctx; g++) *reads += nr[g];
    return KC_OK;
}

// inputMode=exact: the reference's chunks (ExactChunker, GetChunkSize with
// the ctx's gpuMemoryLimit) through kc_count_chunk.
static kc_status file_exact(kc_ctx* c, const char* path, int64_t L, uint64_t* reads) {
    const int64_t limit = c->cfg.gpu_memory_limit ? (int64_t)c->cfg.gpu_memory_limit : 100000000;
    const int64_t cs = kc::reference_chunk_size(L, c->k, limit);
    kc::ExactChunker ch(path, L);
    std::vector<char> buf;
    while (!ch.done()) {
        const int64_t n = ch.next(cs, buf);
        if (n > 0 && n >= L) {  // KMerCounter.cpp:130
            kc_status s = kc_count_chunk(c, buf.data(), n, L);
            if (s) return s;
            *reads += (uint64_t)(n / L);
        }
    }
    return KC_OK;
}

extern "C" kc_status kc_count_file(kc_ctx* const* ctxs, uint32_t n_ctx, const char* path, int64_t L, uint32_t mode,
                                   uint64_t* n_reads) {
    if (!ctxs || n_ctx == 0 || !path || mode > KC_INPUT_EXACT) return KC_ERR_ARG;
    for (uint32_t g = 0; g < n_ctx; g++)
        if (!ctxs[g] || ctxs[g]->k != ctxs[0]->k) return KC_ERR_ARG;
    kc_ctx* c0 = ctxs[0];
    const bool var = (c0->cfg.flags & KC_FLAG_VARLEN) != 0;
    if (n_reads) *n_reads = 0;
    if (L == 0) L = var ? c0->cfg.line_length : kc::file_line2_length(path);
    // reads shorter than k have no windows (the reference's CLI skips such files)
    if (L < c0->k) return KC_OK;
    kc_status s = check_line(c0, L);
    if (s) return s;
    for (uint32_t g = 0; g < n_ctx; g++) {  // chunks accumulated by kc_count_chunk are counted first
        HIPCHK(ctxs[g], hipSetDevice(ctxs[g]->cfg.device));
        if ((s = chunk_acc_flush(ctxs[g]))) return s;
    }
    uint64_t reads = 0;
    kc_ctx* failed = nullptr;
    if (mode == KC_INPUT_EXACT) {
        if (var) return fail(c0, KC_ERR_ARG, "variable-length reads have no reference chunk form");
        s = file_exact(c0, path, L, &reads);
    } else if (mode == KC_INPUT_FASTQ || var) {
        s = file_blocks(ctxs, n_ctx, path, L, true, &reads, &failed);
    } else {
        // auto: GPU decode; a malformed block sends the whole file to the
        // reference chunker. The file is read once when its reads fit every
        // context's checkpoint room (rolled back on a malformed block), else
        // it is validated first.
        struct stat sb;
        if (stat(path, &sb) != 0) return fail(c0, KC_ERR_IO, "cannot stat %s: %s", path, strerror(errno));
        const uint64_t est = (uint64_t)sb.st_size / (uint64_t)(2 * L + 6) + 1;  // records are >= 2L + 6 bytes
        bool once = true;
        for (uint32_t g = 0; g < n_ctx; g++) {
            kc_ctx* c = ctxs[g];
            c->ckpt = true;
            const uint64_t room = pend_room(c, L);
            c->ckpt = false;
            if ((c->pend_reads && (c->pend_L != L || c->pend_var)) || (c->pend_L == L ? c->pend_reads : 0) + est > room)
                once = false;
        }
        bool exact = false;
        if (once) {
            for (uint32_t g = 0; g < n_ctx; g++)
                if ((s = kc_checkpoint(ctxs[g]))) return s;
            s = file_blocks(ctxs, n_ctx, path, L, true, &reads, &failed);
            if (s == KC_ERR_FORMAT) {
                for (uint32_t g = 0; g < n_ctx; g++) {
                    kc_status r = kc_rollback(ctxs[g]);
                    if (r) return r;
                }
                exact = true;
                reads = 0;
            } else {
                for (uint32_t g = 0; g < n_ctx; g++) kc_commit(ctxs[g]);
            }
        } else {
            uint64_t dummy = 0;
            s = file_blocks(ctxs, n_ctx, path, L, false, &dummy, &failed);
            if (s == KC_ERR_FORMAT) {
                exact = true;
            } else if (!s) {
                s = file_blocks(ctxs, n_ctx, path, L, true, &reads, &failed);
            }
        }
        if (exact) s = file_exact(c0, path, L, &reads);
    }
    if (s) {
        if (failed && failed != c0) c0->err = failed->err;  // the caller reads ctxs[0]'s message
        return s;
    }
    if (n_reads) *n_reads = reads;
    return KC_OK;
}

kc_status kc_checkpoint(kc_ctx* c) {
    if (!c) return KC_ERR_ARG;
    if (c->finished) return fail(c, KC_ERR_STATE, "kc_finish was called; kc_reset first");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    kc_status s = chunk_acc_flush(c);  // accumulated chunks are counted before the checkpoint
    if (s) return s;
    s = sync_stats(c);
    if (s) return s;
    c->ckpt = true;
    c->ckpt_reads = c->pend_reads;
    c->ckpt_flushes = c->flushes;
    c->ckpt_st_reads = c->st.reads;
    c->ckpt_st_windows = c->st.windows;
    memcpy(c->ckpt_stats, c->stats_h, sizeof(c->ckpt_stats));
    return KC_OK;
}

kc_status kc_rollback(kc_ctx* c) {
    if (!c) return KC_ERR_ARG;
    if (!c->ckpt) return fail(c, KC_ERR_STATE, "no checkpoint");
    c->ckpt = false;
    if (c->flushes != c->ckpt_flushes || c->finished)
        return fail(c, KC_ERR_STATE, "reads were counted since the checkpoint: it cannot be rolled back");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    c->pend_reads = c->ckpt_reads;
    if (c->pend_reads == 0) c->pend_sparse = false;  // (rows kept keep their lengths)
    c->acc_n = 0;  // chunks accumulated since (kc_checkpoint flushed the accumulator) are forgotten too
    c->st.reads = c->ckpt_st_reads;
    c->st.windows = c->ckpt_st_windows;
    HIPCHK(c, hipMemcpyAsync(c->stats, c->ckpt_stats, sizeof(c->ckpt_stats), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    memcpy(c->stats_h, c->ckpt_stats, sizeof(c->ckpt_stats));
    return KC_OK;
}

kc_status kc_commit(kc_ctx* c) {
    if (!c) return KC_ERR_ARG;
    c->ckpt = false;
    return KC_OK;
}

static kc_status sort_reduce_pack(kc_ctx* c, uint64_t out_cap, uint64_t n, bool dups, uint64_t* n_out);
static kc_status reduce_pack(kc_ctx* c, uint64_t out_cap, uint64_t n, int which, bool dups, uint64_t* n_out);

// Sorted finish of the partition engine (one batch, every key counted in LDS):
// the records of each P5 pass form one key-ordered segment; the descriptors
// (bucket << 48 | first key fraction) are sorted, their lengths scanned into
// output offsets, and seg_sort sorts every segment into place. Key 0, the
// smallest key, goes first. No global radix sort.
static kc_status finish_part_sorted(kc_ctx* c, uint64_t ndesc, uint64_t* n_out) {
    kc_status s;
    const int W = c->W;
    const uint64_t nrec = c->rec_n;
    const bool key0 = c->stats_h[ST_KEY0_PRESENT] != 0;
    const uint64_t off0 = key0 ? 1 : 0;
    const uint64_t n = nrec + off0;
    const uint64_t out_cap = n + 1;
    if ((s = ensure(c, c->fin_keys[0], (size_t)W * out_cap * 8)) || (s = ensure(c, c->fin_cnts[0], out_cap * 4)))
        return s;
    uint64_t* k0 = (uint64_t*)c->fin_keys[0].p;
    uint32_t* c0 = (uint32_t*)c->fin_cnts[0].p;
    if (ndesc) {
        if ((s = ensure(c, c->desc_k2, ndesc * 8)) || (s = ensure(c, c->desc_v, ndesc * 4)) ||
            (s = ensure(c, c->desc_v2, ndesc * 4)) || (s = ensure(c, c->desc_lens, ndesc * 8)) ||
            (s = ensure(c, c->desc_offs, ndesc * 8)) || (s = ensure(c, c->rle_tmp, scan_tmp_elems(ndesc) * 8)))
            return s;
        // KC_TRACE: each phase synchronised and timed
        double tp = kc::trace_on() ? kc::now_s() : 0;
        auto phase = [&](const char* what) {
            if (!kc::trace_on()) return;
            if (hipStreamSynchronize(c->stream) != hipSuccess) return;
            const double t = kc::now_s();
            kc::trace("finish_part_sorted %s: %.3f ms", what, (t - tp) * 1e3);
            tp = t;
        };
        phase("buffers");
        HIPCHK(c, launch_iota_u32((uint32_t*)c->desc_v.p, ndesc, c->stream));
        int which = 0;
        if ((s = sort_records(c, (uint64_t*)c->desc_key.p, (uint64_t*)c->desc_k2.p, (uint32_t*)c->desc_v.p,
                              (uint32_t*)c->desc_v2.p, ndesc, ndesc, &which, 1)))
            return s;
        phase("descriptor sort");
        const uint32_t* order = (const uint32_t*)(which ? c->desc_v2.p : c->desc_v.p);
        HIPCHK(c, launch_desc_prep(order, (const uint32_t*)c->desc_len.p, ndesc, (uint64_t*)c->desc_lens.p,
                                   c->stream));
        HIPCHK(c, launch_scan_u64((const uint64_t*)c->desc_lens.p, (uint64_t*)c->desc_offs.p, ndesc,
                                  (uint64_t*)c->rle_tmp.p, c->stream));
        // LSD fallback list (u32 per descriptor + count) in the free sort scratch
        uint32_t* fb = (uint32_t*)c->desc_k2.p;
        uint64_t* fb_n = (uint64_t*)c->desc_lens.p;  // desc_lens is consumed by the scan above
        if ((s = ensure(c, c->desc_fb, ndesc * 4 + 16))) return s;
        fb = (uint32_t*)c->desc_fb.p;
        // sorted straight into the packed output, after the key-0 record
        if ((s = ensure_pooled(c, c->fin_packed, (size_t)n * c->rs + 16))) return s;
        phase("descriptor scan");
        HIPCHK(c, launch_seg_sort(W, c->rec_keys, c->rec_cnts, c->rec_cap, order, (const uint64_t*)c->desc_start.p,
                                  (const uint32_t*)c->desc_len.p, (const uint64_t*)c->desc_offs.p, ndesc, k0 + off0,
                                  c0 + off0, out_cap, c->stats, fb, fb_n, c->n_cu, c->stream,
                                  (char*)c->fin_packed.p + off0 * c->rs,
                                  (const uint64_t*)(which ? c->desc_k2.p : c->desc_key.p)));
        phase("segment sort");
    }
    if ((s = ensure_pooled(c, c->fin_packed, (size_t)n * c->rs + 16))) return s;
    // record 0: key 0^W (all-zero words) and its count (kept alive until the
    // stream is synchronised below)
    std::vector<uint32_t> r0((size_t)c->rs / 4, 0u);
    if (key0) {
        r0.back() = (uint32_t)c->stats_h[ST_KEY0];
        HIPCHK(c, hipMemcpyAsync(c->fin_packed.p, r0.data(), c->rs, hipMemcpyHostToDevice, c->stream));
    }
    if ((s = sync_stats(c))) return s;
    if (c->stats_h[ST_ERR] & ERR_SEG_TOO_LONG) return fail(c, KC_ERR_INTERNAL, "segment longer than its LDS sort");
    *n_out = n;
    return KC_OK;
}

// Finish whenever an skm batch contributed: the P5 records (+ global-table
// records + key 0) are grouped by their first 8 bases (word0 >> 48) with the
// rp_* passes (counts as payload), every group is sorted in LDS by seg_sort_k,
// equal keys (several batches, the global table) are summed, then packed. A
// group longer than seg_sort's capacity (skewed keys) or a small record set
// takes the global radix sort instead.
static kc_status finish_skm(kc_ctx* c, uint64_t* n_out) {
    kc_status s;
    const int W = c->W;
    const uint64_t nrec = c->rec_n;
    const uint64_t claimed = c->stats_h[ST_CLAIMED];
    if ((s = grow_records(c, nrec + claimed + 1))) return s;
    if ((s = ensure(c, c->fin_misc, (2 * W + 2 + compact_tmp_elems()) * 8))) return s;
    uint64_t* cursor = (uint64_t*)c->fin_misc.p + 2 * W;
    uint64_t* longest = cursor + 1 + compact_tmp_elems();
    uint64_t t = 0;
    if (claimed) {
        HIPCHK(c, launch_compact(W, c->table, c->cap, c->rec_keys + nrec, c->rec_cnts + nrec, c->rec_cap, cursor,
                                 cursor + 1, c->stream));
        HIPCHK(c, hipMemcpyAsync(&t, cursor, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    const uint64_t cur = nrec + t;  // (kept alive until the stream is synchronised below)
    HIPCHK(c, hipMemcpyAsync(cursor, &cur, 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_append_key0(W, c->rec_keys, c->rec_cnts, c->rec_cap, cursor, c->stats, c->stream));
    uint64_t n = 0;
    HIPCHK(c, hipMemcpyAsync(&n, cursor, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const bool dups = c->batches > 1 || t > 0;
    const uint64_t out_cap = n + 1;
    for (int i = 0; i < 2; i++) {
        if ((s = ensure(c, c->fin_keys[i], (size_t)W * out_cap * 8)) || (s = ensure(c, c->fin_cnts[i], out_cap * 4)))
            return s;
    }
    uint64_t* k0 = (uint64_t*)c->fin_keys[0].p;
    uint32_t* c0 = (uint32_t*)c->fin_cnts[0].p;
    const uint32_t nb = 1u << kBucketBits;
    bool grouped = n >= nb && n <= c->key_cap && !test_hook("KC_NO_SEGSORT");
    if (grouped) {
        // only the skm engine wrote records since the reset: P5 wrote their
        // first grouping digit (rec_dig), the table's and key 0's (appended
        // above) are added here, and the first pass reads 1 B per record
        const bool dig1 = c->engines_used == 1 && c->rec_dig && !test_hook("KC_NO_REC_DIG");
        if (dig1 && n > nrec)
            HIPCHK(c, launch_key_digits(c->rec_keys, nrec, n, 48, c->rec_dig, c->stream));
        double gm[2] = {0, 0};
        if ((s = group16(c, W, true, c->rec_keys, c->rec_cap, c->rec_cnts, (uint64_t*)c->fin_keys[1].p, out_cap,
                         (uint32_t*)c->fin_cnts[1].p, c->digs, n, gm, dig1 ? c->rec_dig : nullptr)))
            return s;
        c->finish_group_ms += gm[0] + gm[1];
        if ((s = ensure(c, c->part_starts, ((size_t)nb + 1) * 8)) || (s = ensure(c, c->desc_v, (size_t)nb * 4)) ||
            (s = ensure(c, c->desc_len, (size_t)nb * 4)) || (s = ensure(c, c->desc_fb, (size_t)nb * 4 + 16)))
            return s;
        HIPCHK(c, launch_bucket_bounds(W, c->rec_keys, c->rec_cap, n, kBucketBits, (uint64_t*)c->part_starts.p,
                                       c->stream));
        // the groups' descriptors (digit: word0 bits 36..47, the 12 bits below
        // the 16-bit group prefix) built on the device; only the longest
        // group's length comes back
        HIPCHK(c, hipMemsetAsync(longest, 0, 8, c->stream));
        HIPCHK(c, launch_group_desc((const uint64_t*)c->part_starts.p, nb, 36u, (uint32_t*)c->desc_v.p,
                                    (uint32_t*)c->desc_len.p, longest, c->stream));
        uint64_t mx = 0;
        HIPCHK(c, hipMemcpyAsync(&mx, longest, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (mx > (uint64_t)seg_sort_cap(W)) grouped = false;
    }
    if (grouped) {
        uint64_t* fb_n = (uint64_t*)((char*)c->desc_fb.p + (size_t)nb * 4);
        // one batch, no table records: keys are distinct, so the groups are
        // sorted straight into the packed output
        if (!dups && (s = ensure(c, c->fin_packed, (size_t)n * c->rs + 16))) return s;
        HIPCHK(c, launch_seg_sort(W, c->rec_keys, c->rec_cnts, c->rec_cap, (const uint32_t*)c->desc_v.p,
                                  (const uint64_t*)c->part_starts.p, (const uint32_t*)c->desc_len.p,
                                  (const uint64_t*)c->part_starts.p, nb, k0, c0, out_cap, c->stats,
                                  (uint32_t*)c->desc_fb.p, fb_n, c->n_cu, c->stream, dups ? nullptr : c->fin_packed.p));
        if ((s = sync_stats(c))) return s;
        if (c->stats_h[ST_ERR] & ERR_SEG_TOO_LONG) return fail(c, KC_ERR_INTERNAL, "segment longer than its LDS sort");
        if (!dups) {
            *n_out = n;
            return KC_OK;
        }
        return reduce_pack(c, out_cap, n, 0, dups, n_out);
    }
    if (n) {
        for (int j = 0; j < W; j++)
            HIPCHK(c, hipMemcpyAsync(k0 + (size_t)j * out_cap, c->rec_keys + (size_t)j * c->rec_cap, n * 8,
                                     hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c0, c->rec_cnts, n * 4, hipMemcpyDeviceToDevice, c->stream));
    }
    return sort_reduce_pack(c, out_cap, n, dups, n_out);
}

// Finish of the partition engine: LDS records + fallback-table records + key 0
// -> radix sort -> (sum duplicates when several batches or the fallback table
// contributed) -> pack.
static kc_status finish_part(kc_ctx* c, uint64_t* n_out) {
    if (c->skm_used) return finish_skm(c, n_out);
    kc_status s;
    const int W = c->W;
    const uint64_t nrec = c->rec_n;
    const uint64_t claimed = c->stats_h[ST_CLAIMED];
    const uint64_t ndesc = c->stats_h[ST_DESC_FILL];
    kc::trace("finish_part: %llu records, %llu batches, %llu claimed, %zu host runs, %llu descriptors",
              (unsigned long long)nrec, (unsigned long long)c->batches, (unsigned long long)claimed, c->runs.size(),
              (unsigned long long)ndesc);
    if (c->batches <= 1 && claimed == 0 && c->runs.empty() && ndesc <= kDescCap && !test_hook("KC_NO_SEGSORT"))
        return finish_part_sorted(c, ndesc, n_out);
    const uint64_t out_cap = nrec + claimed + 1;
    for (int i = 0; i < 2; i++) {
        if ((s = ensure(c, c->fin_keys[i], (size_t)W * out_cap * 8)) || (s = ensure(c, c->fin_cnts[i], out_cap * 4)))
            return s;
    }
    if ((s = ensure(c, c->fin_misc, (2 * W + 1 + compact_tmp_elems()) * 8))) return s;
    uint64_t* k0 = (uint64_t*)c->fin_keys[0].p;
    uint32_t* c0 = (uint32_t*)c->fin_cnts[0].p;
    uint64_t* cursor = (uint64_t*)c->fin_misc.p + 2 * W;
    if (nrec) {
        for (int j = 0; j < W; j++)
            HIPCHK(c, hipMemcpyAsync(k0 + (size_t)j * out_cap, c->rec_keys + (size_t)j * c->rec_cap, nrec * 8,
                                     hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c0, c->rec_cnts, nrec * 4, hipMemcpyDeviceToDevice, c->stream));
    }
    uint64_t t = 0;
    if (claimed) {
        HIPCHK(c, launch_compact(W, c->table, c->cap, k0 + nrec, c0 + nrec, out_cap, cursor, cursor + 1, c->stream));
        HIPCHK(c, hipMemcpyAsync(&t, cursor, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    uint64_t cur = nrec + t;
    HIPCHK(c, hipMemcpyAsync(cursor, &cur, 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_append_key0(W, k0, c0, out_cap, cursor, c->stats, c->stream));
    uint64_t n = 0;
    HIPCHK(c, hipMemcpyAsync(&n, cursor, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return sort_reduce_pack(c, out_cap, n, c->batches > 1 || t > 0, n_out);
}

static kc_status reduce_pack(kc_ctx* c, uint64_t out_cap, uint64_t n, int which, bool dups, uint64_t* n_out);

// fin_keys[0]/fin_cnts[0] hold n records at stride out_cap: radix sort, sum
// equal keys when `dups` may exist, pack into fin_packed.
static kc_status sort_reduce_pack(kc_ctx* c, uint64_t out_cap, uint64_t n, bool dups, uint64_t* n_out) {
    kc_status s;
    uint64_t* k0 = (uint64_t*)c->fin_keys[0].p;
    uint32_t* c0 = (uint32_t*)c->fin_cnts[0].p;
    int which = 0;
    if ((s = sort_records(c, k0, (uint64_t*)c->fin_keys[1].p, c0, (uint32_t*)c->fin_cnts[1].p, out_cap, n, &which)))
        return s;
    return reduce_pack(c, out_cap, n, which, dups, n_out);
}

// fin_keys[which]/fin_cnts[which] hold n sorted records (equal keys adjacent):
// sum equal keys (segmented reduce) when `dups`, pack into fin_packed.
static kc_status reduce_pack(kc_ctx* c, uint64_t out_cap, uint64_t n, int which, bool dups, uint64_t* n_out) {
    kc_status s;
    const int W = c->W;
    if (dups && n > 1) {
        uint64_t* ks = (uint64_t*)c->fin_keys[which].p;
        uint32_t* cs = (uint32_t*)c->fin_cnts[which].p;
        uint64_t* ko = (uint64_t*)c->fin_keys[which ^ 1].p;
        uint32_t* co = (uint32_t*)c->fin_cnts[which ^ 1].p;
        if ((s = ensure(c, c->rle_flags, n * 4)) || (s = ensure(c, c->rle_pos, n * 4)) ||
            (s = ensure(c, c->rle_tmp, scan_tmp_elems(n) * 4)))
            return s;
        HIPCHK(c, launch_rle_heads(W, ks, out_cap, n, (uint32_t*)c->rle_flags.p, c->stream));
        HIPCHK(c, launch_scan_u32((uint32_t*)c->rle_flags.p, (uint32_t*)c->rle_pos.p, n, (uint32_t*)c->rle_tmp.p,
                                  c->stream));
        uint32_t last[2];
        HIPCHK(c, hipMemcpyAsync(&last[0], (uint32_t*)c->rle_pos.p + (n - 1), 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(&last[1], (uint32_t*)c->rle_flags.p + (n - 1), 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemsetAsync(co, 0, n * 4, c->stream));
        HIPCHK(c, launch_reduce_add(W, ks, out_cap, cs, n, (uint32_t*)c->rle_flags.p, (uint32_t*)c->rle_pos.p, ko,
                                    out_cap, co, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        n = (uint64_t)last[0] + last[1];
        which ^= 1;
    }
    if ((s = ensure(c, c->fin_packed, (size_t)n * c->rs + 16))) return s;
    HIPCHK(c, launch_pack(W, (uint64_t*)c->fin_keys[which].p, out_cap, (uint32_t*)c->fin_cnts[which].p, n,
                          c->fin_packed.p, c->stream));
    *n_out = n;
    return KC_OK;
}

// Table engine: the global table compacted, radix-sorted and packed into
// fin_packed (key 0 first when present).
static kc_status finish_table(kc_ctx* c, uint64_t* n_out) {
    kc_status s;
    const int W = c->W;
    uint64_t out_cap = c->stats_h[ST_CLAIMED] + 1;
    for (int i = 0; i < 2; i++) {
        if ((s = ensure(c, c->fin_keys[i], (size_t)W * out_cap * 8)) || (s = ensure(c, c->fin_cnts[i], out_cap * 4)))
            return s;
    }
    if ((s = ensure(c, c->fin_misc, (2 * W + 1 + compact_tmp_elems()) * 8))) return s;
    uint64_t* cursor = (uint64_t*)c->fin_misc.p + 2 * W;
    HIPCHK(c, launch_compact(W, c->table, c->cap, (uint64_t*)c->fin_keys[0].p, (uint32_t*)c->fin_cnts[0].p, out_cap,
                             cursor, cursor + 1, c->stream));
    HIPCHK(c, launch_append_key0(W, (uint64_t*)c->fin_keys[0].p, (uint32_t*)c->fin_cnts[0].p, out_cap, cursor,
                                 c->stats, c->stream));
    uint64_t n = 0;
    HIPCHK(c, hipMemcpyAsync(&n, cursor, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (n > out_cap) return fail(c, KC_ERR_INTERNAL, "compaction found %llu records, expected <= %llu",
                                 (unsigned long long)n, (unsigned long long)out_cap);
    int which = 0;
    // note: sort_records re-uses fin_misc for the key bits (cursor already read)
    if ((s = sort_records(c, (uint64_t*)c->fin_keys[0].p, (uint64_t*)c->fin_keys[1].p, (uint32_t*)c->fin_cnts[0].p,
                          (uint32_t*)c->fin_cnts[1].p, out_cap, n, &which)))
        return s;
    if ((s = ensure(c, c->fin_packed, (size_t)n * c->rs + 16))) return s;
    HIPCHK(c, launch_pack(W, (uint64_t*)c->fin_keys[which].p, out_cap, (uint32_t*)c->fin_cnts[which].p, n,
                          c->fin_packed.p, c->stream));
    *n_out = n;
    return KC_OK;
}

kc_status kc_finish(kc_ctx* c, uint64_t* n_records) {
    if (!c) return KC_ERR_ARG;
    if (c->finished) {
        if (n_records) *n_records = c->n_records;
        return KC_OK;
    }
    HIPCHK(c, hipSetDevice(c->cfg.device));
    kc_status s;
    c->ckpt = false;
    if (c->acc_t[3] > 0) {
        kc::trace("chunk calls %.0f: host copy %.3f ms, buffer waits %.3f ms, flushes %.3f ms", c->acc_t[3],
                  c->acc_t[0] * 1e3, c->acc_t[1] * 1e3, c->acc_t[2] * 1e3);
        for (double& x : c->acc_t) x = 0;
    }
    if ((s = pend_flush(c))) return s;
    if ((s = sync_stats(c))) return s;
    if (c->stats_h[ST_SPILL_FILL] > 0 && (s = flush_spill(c))) return s;
    // the table run: the engines' records (or the global table) sorted into fin_packed
    // (own events: the grouping passes inside record ev0..ev2 themselves)
    HIPCHK(c, hipEventRecord(c->evf[0], c->stream));
    uint64_t n = 0;
    if ((s = c->part ? finish_part(c, &n) : finish_table(c, &n))) return s;
    HIPCHK(c, hipEventRecord(c->evf[1], c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float tf = 0.f;
    HIPCHK(c, hipEventElapsedTime(&tf, c->evf[0], c->evf[1]));
    c->st.finish_ms += tf;
    c->st.table_used = c->stats_h[ST_CLAIMED];
    if (c->dev_runs.size() == 1 && n == 0) {
        // one sorted run and no table run (key-range passes, one direct
        // batch): the run is the output, its buffer becomes fin_packed
        if (c->fin_packed.p) c->run_pool.push_back(c->fin_packed);
        c->fin_packed = c->dev_runs[0];
        n = c->dev_run_n[0];
        c->dev_runs.clear();
        c->dev_run_n.clear();
    }
    if (!c->dev_runs.empty()) {
        // sorted runs in HBM (cut runs, spill runs): the table run joins them
        // (taking over fin_packed's buffer), one merge of all
        std::vector<std::pair<const void*, uint64_t>> runs;
        for (size_t r = 0; r < c->dev_runs.size(); r++) runs.push_back({c->dev_runs[r].p, c->dev_run_n[r]});
        DevBuf table_run;
        if (n) {
            table_run = c->fin_packed;
            c->fin_packed = DevBuf();
            if (!c->run_pool.empty()) {
                c->fin_packed = c->run_pool.back();
                c->run_pool.pop_back();
            }
            runs.push_back({table_run.p, n});
        }
        const double tm = kc::trace_on() ? kc::now_s() : 0;
        s = merge_runs_packed(c, runs);
        kc::trace("merge of %zu runs: %.3f ms", runs.size(), (kc::now_s() - tm) * 1e3);
        if (table_run.p) c->run_pool.push_back(table_run);
        release_dev_runs(c, false);
        if (s) return s;
        if (n_records) *n_records = c->n_records;
        return KC_OK;
    }
    c->n_records = n;
    c->finished = true;
    c->st.output_records = n;
    if (n_records) *n_records = n;
    return KC_OK;
}

kc_status kc_copy_records(kc_ctx* c, void* dst, uint64_t dst_bytes) {
    if (!c || !dst) return KC_ERR_ARG;
    if (!c->finished) return fail(c, KC_ERR_STATE, "call kc_finish first");
    if (!c->runs.empty()) return fail(c, KC_ERR_STATE, "spill runs exist: use kc_write_output");
    uint64_t bytes = c->n_records * c->rs;
    if (dst_bytes < bytes) return fail(c, KC_ERR_ARG, "destination holds %llu bytes, need %llu",
                                       (unsigned long long)dst_bytes, (unsigned long long)bytes);
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if (bytes) {
        HIPCHK(c, hipMemcpyAsync(dst, c->fin_packed.p, bytes, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return KC_OK;
}

kc_status kc_device_records(kc_ctx* c, const void** d_records, uint64_t* n_bytes) {
    if (!c || !d_records || !n_bytes) return KC_ERR_ARG;
    if (!c->finished) return fail(c, KC_ERR_STATE, "call kc_finish first");
    *d_records = c->fin_packed.p;
    *n_bytes = c->n_records * c->rs;
    return KC_OK;
}

// The finished table run (SortedKMerFile bytes) to host memory through the
// pinned ring, the pieces copied out by the pool while the next DMA runs.
static kc_status table_run_to_host(kc_ctx* c, std::vector<uint8_t>* mem) {
    const uint64_t bytes = c->n_records * c->rs;
    mem->resize(bytes);
    if (!bytes) return KC_OK;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    kc_status s = stage_init(c);
    if (s) return s;
    uint8_t* dst = mem->data();
    HIPCHK(c, c->ring->download(c->fin_packed.p, bytes, c->stream, [&](const char* p, size_t n, size_t off) {
        kc::par_memcpy(c->pool, dst + off, p, n);
        return true;
    }));
    return KC_OK;
}

// The finished table run into a file at byte `at` (`whole`: the file is
// exactly the run, as after truncating it — the reference appends,
// KMerFileMerger.cpp:129): device -> pinned slot DMAs overlap the writes of
// the previous slot. An existing file is not truncated first but overwritten
// in place and cut to size at the end (truncating a cached file frees its
// pages, ~60 ms per GB, and the writes then allocate them again); the range
// is allocated up front (fallocate), the writes go out in 8 MiB pieces.
static kc_status table_run_to_file(kc_ctx* c, const char* path, uint64_t at = 0, bool whole = true) {
    const uint64_t bytes = c->n_records * c->rs;
    const double t0 = kc::trace_on() ? kc::now_s() : 0;
    int fd = open(path, O_CREAT | O_WRONLY, 0644);
    if (fd < 0) return fail(c, KC_ERR_IO, "cannot open output file %s: %s", path, strerror(errno));
    // the range is reserved up front: a full filesystem fails here, by name,
    // before any byte moves (filesystems without fallocate just write)
    if (bytes && fallocate(fd, 0, (off_t)at, (off_t)bytes) != 0 && errno != EOPNOTSUPP && errno != ENOSYS) {
        const int e = errno;
        close(fd);
        return fail(c, KC_ERR_IO, "cannot reserve %llu bytes at %llu in %s: %s", (unsigned long long)bytes,
                    (unsigned long long)at, path, strerror(e));
    }
    if (kc::trace_on()) kc::trace("output open + fallocate %.3f ms", (kc::now_s() - t0) * 1e3);
    kc_status s = KC_OK;
    if (bytes) {
        HIPCHK(c, hipSetDevice(c->cfg.device));
        if ((s = stage_init(c))) {
            close(fd);
            return s;
        }
        int werr = 0;
        uint64_t wat = 0;
        hipError_t e = c->ring->download(c->fin_packed.p, bytes, c->stream, [&](const char* p, size_t n, size_t off) {
            size_t done = 0;
            while (done < n) {
                const size_t piece = std::min((size_t)8 << 20, n - done);
                ssize_t w = pwrite(fd, p + done, piece, (off_t)(at + off + done));
                if (w < 0 && errno == EINTR) continue;
                if (w <= 0) {
                    werr = w < 0 ? errno : ENOSPC;  // a 0-byte write: no room
                    wat = at + off + done;
                    return false;
                }
                done += (size_t)w;
            }
            return true;
        });
        if (e == hipErrorUnknown)
            s = fail(c, KC_ERR_IO, "write to %s failed at byte %llu of %llu: %s", path, (unsigned long long)wat,
                     (unsigned long long)(at + bytes), strerror(werr));
        else if (e != hipSuccess) s = fail(c, KC_ERR_HIP, "output copy: %s", hipGetErrorString(e));
    }
    if (!s && whole && ftruncate(fd, (off_t)(at + bytes)) != 0)
        s = fail(c, KC_ERR_IO, "cannot size %s: %s", path, strerror(errno));
    if (close(fd) != 0 && !s) s = fail(c, KC_ERR_IO, "cannot close %s: %s", path, strerror(errno));
    if (kc::trace_on()) kc::trace("output %llu bytes in %.3f ms", (unsigned long long)bytes, (kc::now_s() - t0) * 1e3);
    return s;
}

kc_status kc_write_output(kc_ctx* c, const char* path, uint32_t fan_in, uint32_t threads) {
    if (!c || !path) return KC_ERR_ARG;
    if (!c->finished) return fail(c, KC_ERR_STATE, "call kc_finish first");
    if (c->runs.empty()) return table_run_to_file(c, path);
    std::vector<uint8_t> table_run;
    kc_status s = table_run_to_host(c, &table_run);
    if (s) return s;
    std::vector<RunSource> src;
    RunSource t;
    t.mem = table_run.data();
    t.bytes = table_run.size();
    src.push_back(t);
    for (auto& r : c->runs) {
        RunSource x;
        if (!r.path.empty())
            x.path = r.path;
        else {
            x.mem = r.mem.data();
            x.bytes = r.mem.size();
        }
        src.push_back(x);
    }
    std::string err;
    std::string tmp_prefix = std::string(path) + ".kctmp";
    if (!merge_tree(src, path, c->W, fan_in, threads, tmp_prefix, &err))
        return fail(c, KC_ERR_IO, "%s", err.c_str());
    return KC_OK;
}

kc_status kc_write_output_at(kc_ctx* c, const char* path, uint64_t offset) {
    if (!c || !path) return KC_ERR_ARG;
    if (!c->finished) return fail(c, KC_ERR_STATE, "call kc_finish first");
    if (!c->runs.empty()) return fail(c, KC_ERR_STATE, "spill runs exist: use kc_write_output");
    return table_run_to_file(c, path, offset, false);
}

kc_status kc_write_runs(kc_ctx* c, const char* prefix, uint32_t* n_runs) {
    if (!c || !prefix) return KC_ERR_ARG;
    if (!c->finished) return fail(c, KC_ERR_STATE, "call kc_finish first");
    std::vector<uint8_t> table_run;
    kc_status s = table_run_to_host(c, &table_run);
    if (s) return s;
    uint32_t count = 0;
    auto write_one = [&](const uint8_t* p, size_t bytes, const std::string& from) -> kc_status {
        std::string name = std::string(prefix) + "." + std::to_string(count);
        if (!from.empty()) {
            // copy the temp file
            FILE* in = fopen(from.c_str(), "rb");
            FILE* out = fopen(name.c_str(), "wb");
            if (!in || !out) {
                if (in) fclose(in);
                if (out) fclose(out);
                return fail(c, KC_ERR_IO, "cannot copy run %s to %s: %s", from.c_str(), name.c_str(), strerror(errno));
            }
            std::vector<char> buf(1 << 20);
            size_t got;
            while ((got = fread(buf.data(), 1, buf.size(), in)) > 0) fwrite(buf.data(), 1, got, out);
            fclose(in);
            fclose(out);
        } else {
            FILE* out = fopen(name.c_str(), "wb");
            if (!out) return fail(c, KC_ERR_IO, "cannot write run %s: %s", name.c_str(), strerror(errno));
            size_t w = bytes ? fwrite(p, 1, bytes, out) : 0;
            const int we = errno;
            const int ce = fclose(out) != 0 ? errno : 0;
            if (w != bytes || ce) return fail(c, KC_ERR_IO, "short write %s: %s", name.c_str(), strerror(w != bytes ? we : ce));
        }
        count++;
        return KC_OK;
    };
    if ((s = write_one(table_run.data(), table_run.size(), ""))) return s;
    for (auto& r : c->runs)
        if ((s = write_one(r.mem.data(), r.mem.size(), r.path))) return s;
    if (n_runs) *n_runs = count;
    return KC_OK;
}

kc_status kc_get_stats(const kc_ctx* c, kc_stats* out) {
    if (!c || !out) return KC_ERR_ARG;
    *out = c->st;
    for (int i = 0; i < 5; i++) out->part_ms[i] = c->part_ms[i];
    out->presplit_ms = c->presplit_ms;
    out->presplit_batches = c->presplit_batches;
    out->sorted_run_batches = c->sorted_run_batches;
    out->key_passes = c->key_passes;
    out->batches = c->batches_cut + c->batches;
    out->keys = c->part_keys;
    out->p5_launches = c->p5_launches;
    out->table_capacity = c->cap;
    out->valid_kmers = c->stats_h[ST_VALID];
    out->spill_runs = c->runs_cut + c->runs.size();
    out->engines_used = c->engines_used;
    out->dedup_ms = c->dedup_ms;
    out->dedup_records = c->stats_h[ST_DEDUP];
    out->finish_group_ms = c->finish_group_ms;
    return KC_OK;
}

kc_status kc_merge_files(const char* const* inputs, uint32_t n_inputs, const char* output, int64_t kmer_length,
                         uint32_t fan_in, uint32_t threads) {
    if (!output || kmer_length < 1 || kmer_length > KC_MAX_K || (n_inputs && !inputs)) return KC_ERR_ARG;
    int W = (int)((kmer_length + 31) / 32);
    std::vector<RunSource> src;
    for (uint32_t i = 0; i < n_inputs; i++) {
        RunSource r;
        r.path = inputs[i];
        src.push_back(r);
    }
    std::string err;
    if (!merge_tree(src, output, W, fan_in, threads, std::string(output) + ".kctmp", &err)) return KC_ERR_IO;
    return KC_OK;
}

struct kc_merge_part {
    kc::MergedPart part;
};

kc_status kc_merge_part_create(const char* const* inputs, uint32_t n_inputs, int64_t kmer_length, uint32_t part,
                               uint32_t parts, uint32_t threads, kc_merge_part** out, uint64_t* n_bytes) {
    if (!out || kmer_length < 1 || kmer_length > KC_MAX_K || (n_inputs && !inputs) || parts < 1 || part >= parts)
        return KC_ERR_ARG;
    *out = nullptr;
    const int W = (int)((kmer_length + 31) / 32);
    std::vector<RunSource> src;
    for (uint32_t i = 0; i < n_inputs; i++) {
        if (!inputs[i]) return KC_ERR_ARG;
        RunSource r;
        r.path = inputs[i];
        src.push_back(r);
    }
    std::unique_ptr<kc_merge_part> p(new (std::nothrow) kc_merge_part());
    if (!p) return KC_ERR_NOMEM;
    int e = 0;
    try {
        if (!kc::merge_runs_part(src, W, part, parts, threads ? threads : 1, &p->part, &e)) return KC_ERR_IO;
    } catch (const std::bad_alloc&) {
        return KC_ERR_NOMEM;
    }
    if (n_bytes) *n_bytes = p->part.bytes;
    *out = p.release();
    return KC_OK;
}

kc_status kc_merge_part_write(kc_merge_part* p, const char* output, uint64_t offset, uint64_t file_bytes) {
    if (!p || !output) return KC_ERR_ARG;
    if (file_bytes && offset + p->part.bytes > file_bytes) return KC_ERR_ARG;
    return kc::write_part_at(p->part, output, offset, file_bytes) ? KC_OK : KC_ERR_IO;
}

void kc_merge_part_destroy(kc_merge_part* p) { delete p; }

uint64_t kc_synth_fastq_bytes(const kc_synth_spec* sp) {
    if (!sp) return 0;
    return synth_bytes(sp->first_read, sp->n_reads, sp->read_length, (int)sp->layout);
}

static SynthArgs synth_args(const kc_synth_spec* sp) {
    SynthArgs a;
    a.first = sp->first_read;
    a.n = sp->n_reads;
    a.seed = sp->seed;
    a.genome = sp->genome_length;
    a.L = sp->read_length;
    a.Lmin = sp->min_read_length;
    a.layout = (int)sp->layout;
    double thr = sp->n_rate * 9007199254740992.0;
    a.n_threshold = sp->n_rate <= 0 ? 0 : (thr >= 9007199254740992.0 ? (1ull << 53) : (uint64_t)thr);
    return a;
}

static bool synth_ok(const kc_synth_spec* sp) {
    return sp && sp->read_length > 0 && (sp->genome_length == 0 || sp->genome_length >= (uint64_t)sp->read_length) &&
           sp->min_read_length >= 0 && sp->min_read_length <= sp->read_length && sp->layout <= 1 &&
           (sp->layout == 0 || sp->min_read_length == 0 || sp->min_read_length == sp->read_length);
}

kc_status kc_synth_fastq_host(const kc_synth_spec* sp, char* dst, uint64_t dst_bytes) {
    if (!synth_ok(sp) || !dst) return KC_ERR_ARG;
    if (dst_bytes < kc_synth_fastq_bytes(sp)) return KC_ERR_ARG;
    synth_host(synth_args(sp), dst);
    return KC_OK;
}

kc_status kc_synth_fastq_device(kc_ctx* c, const kc_synth_spec* sp, void** d_out, uint64_t* n_bytes) {
    if (!c || !synth_ok(sp) || !d_out) return KC_ERR_ARG;
    uint64_t bytes = kc_synth_fastq_bytes(sp);
    HIPCHK(c, hipSetDevice(c->cfg.device));
    void* p = nullptr;
    HIPCHK(c, hipMalloc(&p, bytes + 64));
    HIPCHK(c, launch_synth(synth_args(sp), (char*)p, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *d_out = p;
    if (n_bytes) *n_bytes = bytes;
    return KC_OK;
}

kc_status kc_synth_free(kc_ctx* c, void* d_buf) {
    if (!c) return KC_ERR_ARG;
    if (d_buf) HIPCHK(c, hipFree(d_buf));
    return KC_OK;
}

kc_status kc_owner_counts(kc_ctx* c, uint32_t world, uint64_t* counts) {
    if (!c || world == 0 || !counts) return KC_ERR_ARG;
    if (!c->finished) return fail(c, KC_ERR_STATE, "call kc_finish first");
    if (!c->runs.empty()) return fail(c, KC_ERR_STATE, "spill runs exist: the key-space exchange needs one run");
    kc_status s;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if ((s = ensure(c, c->part_starts, ((size_t)world + 1) * 8))) return s;
    HIPCHK(c, launch_owner_bounds(c->fin_packed.p, c->rs, c->n_records, world, (uint64_t*)c->part_starts.p, c->stream));
    std::vector<uint64_t> b(world + 1);
    HIPCHK(c, hipMemcpyAsync(b.data(), c->part_starts.p, (world + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (uint32_t o = 0; o < world; o++) counts[o] = b[o + 1] - b[o];
    return KC_OK;
}

kc_status kc_merge_records_device(kc_ctx* c, const void* d_packed, uint64_t n_records) {
    if (!c || (!d_packed && n_records)) return KC_ERR_ARG;
    if (!c->finished) return fail(c, KC_ERR_STATE, "call kc_finish first");
    if (!c->runs.empty()) return fail(c, KC_ERR_STATE, "spill runs exist");
    kc_status s;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    const uint64_t out_cap = n_records + 1;
    const int W = c->W;
    for (int i = 0; i < 2; i++) {
        if ((s = ensure(c, c->fin_keys[i], (size_t)W * out_cap * 8)) || (s = ensure(c, c->fin_cnts[i], out_cap * 4)))
            return s;
    }
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, launch_unpack(W, d_packed, n_records, (uint64_t*)c->fin_keys[0].p, out_cap,
                            (uint32_t*)c->fin_cnts[0].p, c->stream));
    uint64_t n = 0;
    if ((s = sort_reduce_pack(c, out_cap, n_records, true, &n))) return s;
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float t = 0.f;
    HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
    c->st.finish_ms += t;
    c->n_records = n;
    c->st.output_records = n;
    c->finished = true;
    return KC_OK;
}

}  // extern "C"

// Merges sorted packed runs (each a device pointer + record count; equal keys
// within and across runs allowed) into the ctx's finished table run:
// unpacked side by side into SoA keys, merged pairwise by merge path
// (adjacent runs merge into the same range of the other buffer), equal keys
// summed (u32, wrapping), packed into fin_packed.
static kc_status merge_runs_list(kc_ctx* c, const std::vector<std::pair<const void*, uint64_t>>& runs) {
    const uint32_t nruns = (uint32_t)runs.size();
    std::vector<uint64_t> off(nruns + 1, 0);
    for (uint32_t r = 0; r < nruns; r++) off[r + 1] = off[r] + runs[r].second;
    const uint64_t n = off[nruns];
    kc_status s;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    const uint64_t out_cap = n + 1;
    const int W = c->W;
    for (int i = 0; i < 2; i++) {
        if ((s = ensure(c, c->fin_keys[i], (size_t)W * out_cap * 8)) || (s = ensure(c, c->fin_cnts[i], out_cap * 4)))
            return s;
    }
    if ((s = ensure(c, c->fin_misc, merge_split_elems(n) * 8 + 64))) return s;
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    for (uint32_t r = 0; r < nruns; r++)
        if (runs[r].second)
            HIPCHK(c, launch_unpack(W, runs[r].first, runs[r].second, (uint64_t*)c->fin_keys[0].p + off[r], out_cap,
                                    (uint32_t*)c->fin_cnts[0].p + off[r], c->stream));
    int which = 0;
    std::vector<uint64_t> ro = off;
    while (ro.size() > 2) {
        std::vector<uint64_t> nro;
        const uint64_t* ks = (const uint64_t*)c->fin_keys[which].p;
        const uint32_t* cs = (const uint32_t*)c->fin_cnts[which].p;
        uint64_t* kd = (uint64_t*)c->fin_keys[which ^ 1].p;
        uint32_t* cd = (uint32_t*)c->fin_cnts[which ^ 1].p;
        const size_t nr = ro.size() - 1;
        for (size_t r = 0; r < nr; r += 2) {
            nro.push_back(ro[r]);
            if (r + 1 < nr) {
                const uint64_t a0 = ro[r], na = ro[r + 1] - ro[r], nb = ro[r + 2] - ro[r + 1];
                // the merge kernels take base pointers: offset the SoA columns
                HIPCHK(c, launch_merge(W, ks + a0, cs + a0, out_cap, na, ks + a0 + na, cs + a0 + na, out_cap, nb,
                                       kd + a0, cd + a0, out_cap, (uint64_t*)c->fin_misc.p, c->stream));
            } else {
                const uint64_t a0 = ro[r], na = ro[r + 1] - ro[r];
                for (int j = 0; j < W; j++)
                    HIPCHK(c, hipMemcpyAsync(kd + (size_t)j * out_cap + a0, ks + (size_t)j * out_cap + a0, na * 8,
                                             hipMemcpyDeviceToDevice, c->stream));
                HIPCHK(c, hipMemcpyAsync(cd + a0, cs + a0, na * 4, hipMemcpyDeviceToDevice, c->stream));
            }
        }
        nro.push_back(ro.back());
        ro.swap(nro);
        which ^= 1;
    }
    uint64_t nout = 0;
    if ((s = reduce_pack(c, out_cap, n, which, true, &nout))) return s;
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float t = 0.f;
    HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
    c->st.finish_ms += t;
    c->n_records = nout;
    c->st.output_records = nout;
    c->finished = true;
    return KC_OK;
}

// Sorted runs without repeated keys (kc_finish output, cut runs, slices of
// them) -> the finished table run: pairwise merge path over the packed
// records, level by level (launch_merge_packed), into ping-pong buffers; keys
// present in several runs come out as adjacent records and are summed after
// the last level (SoA segmented reduce). One run is taken as it is.
static kc_status merge_runs_packed(kc_ctx* c, const std::vector<std::pair<const void*, uint64_t>>& runs0) {
    kc_status s;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    std::vector<std::pair<const void*, uint64_t>> runs;
    uint64_t n = 0;
    for (auto& r : runs0)
        if (r.second) {
            runs.push_back(r);
            n += r.second;
        }
    const size_t rs = (size_t)c->rs;
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    if ((s = ensure(c, c->fin_misc, (merge_packed_split_elems(c->W, n) + 8) * 8))) return s;
    uint32_t* dup = (uint32_t*)((uint64_t*)c->fin_misc.p + merge_packed_split_elems(c->W, n) + 2);
    uint64_t* split = (uint64_t*)c->fin_misc.p;
    HIPCHK(c, hipMemsetAsync(dup, 0, 4, c->stream));
    if (runs.size() <= 1) {
        if ((s = ensure_pooled(c, c->fin_packed, n * rs + 16))) return s;
        if (n && runs[0].first != c->fin_packed.p)
            HIPCHK(c, hipMemcpyAsync(c->fin_packed.p, runs[0].first, n * rs, hipMemcpyDeviceToDevice, c->stream));
    } else {
        DevBuf* out[2] = {&c->fin_packed, &c->merge_tmp};
        int lvl = 0;
        while (runs.size() > 1) {
            DevBuf* o = out[lvl & 1];
            if ((s = ensure_pooled(c, *o, n * rs + 16))) return s;
            std::vector<std::pair<const void*, uint64_t>> next;
            uint64_t off = 0;
            for (size_t r = 0; r < runs.size(); r += 2) {
                uint8_t* dst = (uint8_t*)o->p + off * rs;
                if (r + 1 < runs.size()) {
                    HIPCHK(c, launch_merge_packed(c->W, runs[r].first, runs[r].second, runs[r + 1].first,
                                                  runs[r + 1].second, dst, split, dup, c->stream));
                    next.push_back({dst, runs[r].second + runs[r + 1].second});
                } else {
                    HIPCHK(c, hipMemcpyAsync(dst, runs[r].first, runs[r].second * rs, hipMemcpyDeviceToDevice,
                                             c->stream));
                    next.push_back({dst, runs[r].second});
                }
                off += next.back().second;
            }
            runs.swap(next);
            lvl++;
        }
        if (runs[0].first != c->fin_packed.p) std::swap(c->fin_packed, c->merge_tmp);
    }
    uint32_t dup_h = 0;
    HIPCHK(c, hipMemcpyAsync(&dup_h, dup, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    uint64_t nout = n;
    if (dup_h) {
        // keys of several runs: sum them (unpack, segmented reduce, pack)
        const uint64_t out_cap = n + 1;
        const int W = c->W;
        for (int i = 0; i < 2; i++)
            if ((s = ensure(c, c->fin_keys[i], (size_t)W * out_cap * 8)) ||
                (s = ensure(c, c->fin_cnts[i], out_cap * 4)))
                return s;
        HIPCHK(c, launch_unpack(W, c->fin_packed.p, n, (uint64_t*)c->fin_keys[0].p, out_cap,
                                (uint32_t*)c->fin_cnts[0].p, c->stream));
        if ((s = reduce_pack(c, out_cap, n, 0, true, &nout))) return s;
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float t = 0.f;
    HIPCHK(c, hipEventElapsedTime(&t, c->ev0, c->ev1));
    c->st.finish_ms += t;
    c->n_records = nout;
    c->st.output_records = nout;
    c->finished = true;
    return KC_OK;
}

// The records counted so far become a sorted run — the reference's sorted
// spill (sortKmers + reduceKMers + FileDump::dumpKmersToFile,
// GPUHandler.cu:456-468, FileDump.cpp:51-58): finished into packed
// SortedKMerFile records (finish_part), kept in HBM outside the counting
// working set (host memory, as a spill run, when HBM is short), and the
// record state starts empty. kc_finish merges the runs on the device.
static kc_status cut_run(kc_ctx* c) {
    kc_status s;
    // inside a flush of padded / one-pass rows: key 0's presence from the reads
    if (c->var_rlen && (s = recompute_presence(c))) return s;
    if ((s = sync_stats(c))) return s;
    uint64_t n = 0;
    const double t0 = kc::trace_on() ? kc::now_s() : 0;
    if ((s = finish_part(c, &n))) return s;  // fin_packed
    HIPCHK(c, hipStreamSynchronize(c->stream));
    kc::trace("cut_run: %llu records finished in %.3f ms", (unsigned long long)n, (kc::now_s() - t0) * 1e3);
    return keep_finished_run(c, n);
}

// fin_packed (n finished records) becomes a sorted run and the record state
// starts empty
static kc_status keep_finished_run(kc_ctx* c, uint64_t n) {
    const size_t bytes = (size_t)n * c->rs;
    if (n) {
        // the run takes over fin_packed's buffer (no copy); fin_packed gets a
        // pooled buffer back (grown by the next finish if it is short)
        size_t mfree = 0, mtotal = 0;
        if (hipMemGetInfo(&mfree, &mtotal) == hipSuccess && mfree > ((size_t)4 << 30)) {
            DevBuf run = c->fin_packed;
            c->fin_packed = DevBuf();
            if (!c->run_pool.empty()) {
                c->fin_packed = c->run_pool.back();
                c->run_pool.pop_back();
            }
            c->dev_runs.push_back(run);
            c->dev_run_n.push_back(n);
            c->runs_cut++;
        } else {
            HostRun hr;
            hr.records = n;
            hr.mem.resize(bytes);
            HIPCHK(c, hipMemcpyAsync(hr.mem.data(), c->fin_packed.p, bytes, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            c->runs.push_back(std::move(hr));
        }
    }
    // empty record state: records, batch count, table claims, key 0, descriptors
    c->rec_n = 0;
    c->batches_cut += c->batches;
    c->batches = 0;
    c->skm_used = false;
    HIPCHK(c, hipMemsetAsync(c->rec_cursor, 0, 8, c->stream));
    if (c->stats_h[ST_CLAIMED]) HIPCHK(c, hipMemsetAsync(c->table, 0, c->table_bytes, c->stream));
    for (int st : {(int)ST_CLAIMED, (int)ST_KEY0, (int)ST_KEY0_PRESENT, (int)ST_DESC_FILL}) c->stats_h[st] = 0;
    HIPCHK(c, hipMemcpyAsync(c->stats, c->stats_h, ST_N * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return KC_OK;
}

// A run is cut when the records outgrow half the working set (the reference's
// "table capacity < distinct" case, SURVEY §8d cfg 5).
static kc_status cut_run_if_full(kc_ctx* c) {
    const uint64_t M = c->cfg.gpu_memory_limit ? c->cfg.gpu_memory_limit : 100000000ull;
    if (!c->part || c->rec_n * (uint64_t)c->rs <= M / 2) return KC_OK;
    return cut_run(c);
}

static void release_dev_runs(kc_ctx* c, bool free_pool) {
    for (auto& r : c->dev_runs) c->run_pool.push_back(r);
    c->dev_runs.clear();
    c->dev_run_n.clear();
    if (free_pool) {
        for (auto& r : c->run_pool) release(r);
        c->run_pool.clear();
    }
}

extern "C" {

kc_status kc_merge_runs_device(kc_ctx* c, const void* d_packed, const uint64_t* run_counts, uint32_t nruns) {
    if (!c || (nruns && !run_counts)) return KC_ERR_ARG;
    if (!c->finished) return fail(c, KC_ERR_STATE, "call kc_finish first");
    if (!c->runs.empty()) return fail(c, KC_ERR_STATE, "spill runs exist");
    std::vector<std::pair<const void*, uint64_t>> runs;
    uint64_t off = 0;
    for (uint32_t r = 0; r < nruns; r++) {
        runs.push_back({(const uint8_t*)d_packed + off * c->rs, run_counts[r]});
        off += run_counts[r];
    }
    if (off && !d_packed) return KC_ERR_ARG;
    // one run may repeat keys (the SoA path sums them); two or more runs come
    // from finished runs: merged packed, repeated keys summed after the merge
    if (nruns >= 2) return merge_runs_packed(c, runs);
    return merge_runs_list(c, runs);
}

kc_status kc_exchange_contexts(kc_ctx* const* ctxs, uint32_t n) {
    if (!ctxs || n == 0) return KC_ERR_ARG;
    for (uint32_t r = 0; r < n; r++) {
        if (!ctxs[r] || ctxs[r]->W != ctxs[0]->W) return KC_ERR_ARG;
        if (!ctxs[r]->finished) return fail(ctxs[r], KC_ERR_STATE, "call kc_finish first");
        if (!ctxs[r]->runs.empty()) return fail(ctxs[r], KC_ERR_STATE, "spill runs exist");
    }
    const uint64_t rs = (uint64_t)ctxs[0]->rs;
    std::vector<std::vector<uint64_t>> cnt(n, std::vector<uint64_t>(n));
    kc_status s;
    for (uint32_t r = 0; r < n; r++)
        if ((s = kc_owner_counts(ctxs[r], n, cnt[r].data()))) return s;
    // Gather every owner's slices before any merge: a merge overwrites the
    // owner's own packed run, which the other owners still read from.
    std::vector<void*> recv(n, nullptr);
    std::vector<uint64_t> m(n, 0);
    auto release = [&]() {
        for (uint32_t o = 0; o < n; o++)
            if (recv[o]) {
                (void)hipSetDevice(ctxs[o]->cfg.device);
                (void)hipFree(recv[o]);
            }
    };
    for (uint32_t o = 0; o < n; o++) {
        kc_ctx* co = ctxs[o];
        for (uint32_t r = 0; r < n; r++) m[o] += cnt[r][o];
        hipError_t e = hipSetDevice(co->cfg.device);
        if (e == hipSuccess) e = hipMalloc(&recv[o], m[o] * rs + 16);
        uint64_t off = 0;
        for (uint32_t r = 0; r < n && e == hipSuccess; r++) {
            uint64_t src = 0;
            for (uint32_t p = 0; p < o; p++) src += cnt[r][p];
            uint64_t bytes = cnt[r][o] * rs;
            if (bytes)
                e = hipMemcpyPeerAsync((uint8_t*)recv[o] + off, co->cfg.device,
                                       (const uint8_t*)ctxs[r]->fin_packed.p + src * rs, ctxs[r]->cfg.device, bytes,
                                       co->stream);
            off += bytes;
        }
        if (e != hipSuccess) {
            release();
            return fail(co, KC_ERR_HIP, hipGetErrorString(e));
        }
    }
    for (uint32_t o = 0; o < n; o++) {
        hipError_t e = hipSetDevice(ctxs[o]->cfg.device);
        if (e == hipSuccess) e = hipStreamSynchronize(ctxs[o]->stream);
        if (e != hipSuccess) {
            release();
            return fail(ctxs[o], KC_ERR_HIP, hipGetErrorString(e));
        }
    }
    // owner o received one sorted slice from every context, in order; the
    // owners merge concurrently, one host thread each (each context has its
    // own stream and buffers; hipSetDevice is per thread)
    std::vector<kc_status> ms(n, KC_OK);
    auto merge_owner = [&](uint32_t o) {
        std::vector<uint64_t> rc(n);
        for (uint32_t r = 0; r < n; r++) rc[r] = cnt[r][o];
        if (hipSetDevice(ctxs[o]->cfg.device) != hipSuccess) {
            ms[o] = fail(ctxs[o], KC_ERR_HIP, "hipSetDevice(%d)", ctxs[o]->cfg.device);
            return;
        }
        ms[o] = kc_merge_runs_device(ctxs[o], recv[o], rc.data(), n);
    };
    if (n == 1) {
        merge_owner(0);
    } else {
        std::vector<std::thread> th;
        for (uint32_t o = 0; o < n; o++) th.emplace_back(merge_owner, o);
        for (auto& t : th) t.join();
    }
    release();
    for (uint32_t o = 0; o < n; o++)
        if (ms[o]) return ms[o];
    return KC_OK;
}

kc_status kc_gather_contexts(kc_ctx* const* ctxs, uint32_t n) {
    if (!ctxs || n == 0) return KC_ERR_ARG;
    for (uint32_t r = 0; r < n; r++) {
        if (!ctxs[r] || ctxs[r]->W != ctxs[0]->W) return KC_ERR_ARG;
        if (!ctxs[r]->finished) return fail(ctxs[r], KC_ERR_STATE, "call kc_finish first");
        if (!ctxs[r]->runs.empty()) return fail(ctxs[r], KC_ERR_STATE, "host spill runs exist: merge on the host");
    }
    kc_ctx* c0 = ctxs[0];
    const uint64_t rs = (uint64_t)c0->rs;
    uint64_t total = 0;
    for (uint32_t r = 0; r < n; r++) total += ctxs[r]->n_records;
    HIPCHK(c0, hipSetDevice(c0->cfg.device));
    void* recv = nullptr;
    HIPCHK(c0, hipMalloc(&recv, total * rs + 16));
    std::vector<std::pair<const void*, uint64_t>> runs;
    uint64_t off = 0;
    for (uint32_t r = 0; r < n; r++) {
        const uint64_t bytes = ctxs[r]->n_records * rs;
        hipError_t e = bytes ? hipMemcpyPeerAsync((uint8_t*)recv + off * rs, c0->cfg.device, ctxs[r]->fin_packed.p,
                                                  ctxs[r]->cfg.device, bytes, c0->stream)
                             : hipSuccess;
        if (e != hipSuccess) {
            (void)hipFree(recv);
            return fail(c0, KC_ERR_HIP, "gather: %s", hipGetErrorString(e));
        }
        runs.push_back({(uint8_t*)recv + off * rs, ctxs[r]->n_records});
        off += ctxs[r]->n_records;
    }
    hipError_t e = hipStreamSynchronize(c0->stream);
    kc_status s = e == hipSuccess ? merge_runs_packed(c0, runs) : fail(c0, KC_ERR_HIP, "gather: %s", hipGetErrorString(e));
    (void)hipFree(recv);
    return s;
}

kc_status kc_copy_device(kc_ctx* c, void* d_dst, const void* d_src, uint64_t n) {
    if (!c || (n && (!d_dst || !d_src))) return KC_ERR_ARG;
    if (n == 0) return KC_OK;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipMemcpyAsync(d_dst, d_src, n, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return KC_OK;
}

kc_status kc_copy_to_host(kc_ctx* c, void* dst, const void* d_src, uint64_t n) {
    if (!c || (n && (!dst || !d_src))) return KC_ERR_ARG;
    if (n == 0) return KC_OK;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipMemcpyAsync(dst, d_src, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return KC_OK;
}

}  // extern "C"
