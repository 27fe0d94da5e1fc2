// kc_device.h — host-side declarations of the HIP kernels' launch wrappers
// (implemented in kc_kernels.hip, used by kc_api.cpp). Internal to libkc_hip.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdlib.h>

namespace kc {

// Timing ablations (skip a stage; every output after it is invalid) exist only
// in experiment builds (-DKC_EXPERIMENTS, tools/build_variant.sh). The release
// library never reads these variables, so a stray one cannot change a count.
inline int experiment_knob(const char* name) {
#ifdef KC_EXPERIMENTS
    const char* e = getenv(name);
    return e ? atoi(e) : 0;
#else
    (void)name;
    return 0;
#endif
}

// Path-selecting test hooks (KC_NO_P3B, KC_SKM_POOL_CAP, KC_NO_F3, ...):
// they force fallbacks and alternative layouts so the tests can reach them,
// and every one of them gives the same counts. A production caller never
// meets them by accident: the library reads them only when KC_TEST_HOOKS=1
// is set in the environment (tests/conftest.py sets it for the test suite).
inline const char* test_hook(const char* name) {
    static const bool on = [] {
        const char* e = getenv("KC_TEST_HOOKS");
        return e && e[0] == '1' && e[1] == 0;
    }();
    return on ? getenv(name) : nullptr;
}

// Device counters, one uint64 each, in a small device array owned by the ctx.
enum Stat : int {
    ST_VALID = 0,        // valid k-mer windows seen
    ST_KEY0 = 1,         // count of key 0^W (kept outside the table: 0 is the EMPTY key)
    ST_KEY0_PRESENT = 2, // key 0^W must appear in the output (a key-0 window or a hole)
    ST_SPILLED = 3,      // keys appended to the spill buffer
    ST_CLAIMED = 4,      // table slots claimed (= occupied)
    ST_ERR = 5,          // bit set: ERR_* below
    ST_SPILL_FILL = 6,   // next free spill index (may exceed capacity on overflow)
    ST_SPILL2_FILL = 7,  // partition engine P5: keys spilled into the free key buffer
    ST_P5_PASSES = 8,    // P5 sub-range passes emitted (diagnostic)
    ST_P5_ABORTS = 9,    // P5 passes aborted on a full LDS table (diagnostic)
    ST_P5_MAXM = 10,     // largest sub-range split m used (diagnostic)
    ST_DESC_FILL = 11,   // P5 segment descriptors written (may exceed capacity)
    ST_P5_KEYS = 12,     // skm P5 sample launch: keys of the sampled buckets
    ST_DEDUP = 13,       // skm P5a: distinct records listed (raw buckets: their records)
    ST_VHOLE = 14,       // variable-length reads: a read of >= k bases holds a not-ACGT base
    ST_VWIN = 15,        // variable-length reads: windows of the reads' own lengths
    ST_N = 16
};

enum ErrBits : uint64_t {
    ERR_SPILL_OVERFLOW = 1,
    ERR_FQ_NOT_AT = 2,      // record does not start with '@'
    ERR_FQ_NO_PLUS = 4,     // line after the sequence does not start with '+'
    ERR_FQ_SEQ_LEN = 8,     // sequence line length != L
    ERR_FQ_TOO_MANY = 16,   // more records than the index buffer holds
    ERR_FQ_NO_FINAL_NL = 32, // block does not end with '\n'
    ERR_REC_OVERFLOW = 64,   // partition engine: record buffer too small
    ERR_SEG_TOO_LONG = 128,  // seg_sort: a segment longer than its LDS capacity
    ERR_FQ_LIST = 256,       // fused variable-length index: a half held more records than its list (not a
                             // format error: the block is indexed again by the two-pass path)
    ERR_FQ_SPEC = 512        // one-pass index: a chunk's guessed line phase was wrong or not found (not a
                             // format error: the block is indexed again by the two-kernel path)
};

// Slot stride (uint64 words) of the open-addressed table for W key words:
// W=1: {key, count}; W>=2: {key[W], count:u32 | state:u32} padded so that a
// slot never straddles a 64-byte line.
inline int slot_words(int W) { return W == 1 ? 2 : (W <= 3 ? 4 : 8); }

struct CountLaunch {
    const uint8_t* base;      // FASTQ block or stride-L chunk (device)
    const uint64_t* seq_off;  // per-read start offsets, or nullptr for stride mode
    uint64_t read0;           // first read of this launch
    uint64_t n_reads;         // reads in this launch
    int L, k;
    uint64_t* table;
    uint64_t cap;             // slots
    uint64_t* spill;          // SoA: word j of entry i at spill[j*spill_cap + i]
    uint64_t spill_cap;
    uint64_t* stats;          // ST_N counters
    uint32_t probe_limit;
    const uint32_t* codes = nullptr;   // partition engine: reads encoded by kernel E
    const uint16_t* inval = nullptr;   //   (groups_per_read(L) words per read)
    const uint16_t* rlen = nullptr;    // KC_FLAG_VARLEN: each read's own length (<= L), read r at rlen[r]
    uint32_t flo = 0, fhi = 256;       // partition P1/P2: keys with word0 >> 56 in [flo, fhi) only
    bool no_stats = false;             //   (key-range passes after the first: statistics counted once)
};

// E: encode the launch's reads once into 2-bit codes (u32 per 16 bases, first
// base highest) and not-ACGT masks (u16 per 16 bases); read r of the launch at
// r * groups_per_read(L). P1 and P2 read these instead of the FASTQ text.
int groups_per_read(int L);
// stats (may be null): stats[ST_VHOLE] set when a read holds a not-ACGT base
hipError_t launch_encode_reads(const CountLaunch& l, uint32_t* codes, uint16_t* inval, hipStream_t s,
                               uint64_t* stats = nullptr);
// Variable-length reads (KC_FLAG_VARLEN): read r = text [seq_off[r], seq_end[r])
// of at most L bases, encoded as a read of L bases whose positions past its
// own end are not-ACGT with code 0 (no window reaches them; a key's bases past
// the read end read as 0). Sets ERR_FQ_SEQ_LEN for a read longer than L,
// stats[ST_VHOLE] when a read of >= k bases holds a not-ACGT base, adds the
// reads' own windows to stats[ST_VWIN].
// rlen (may be nullptr): each read's own length.
hipError_t launch_encode_reads_var(const uint8_t* base, const uint64_t* seq_off, const uint64_t* seq_end,
                                   uint64_t n_reads, int L, int k, uint32_t* codes, uint16_t* inval, uint16_t* rlen,
                                   uint64_t* stats, hipStream_t s);

// Tile geometry of count_kmers for (L, k); also used to size dynamic LDS.
struct CountGeom {
    int R;          // reads per tile
    int NG;         // 16-base groups per read in LDS
    int raw_stride; // LDS bytes per read of raw text
    size_t lds;     // dynamic LDS bytes
};
CountGeom count_geometry(int L, int k);

hipError_t launch_count_kmers(const CountLaunch& a, int grid_cap, hipStream_t s);

// ---- partition engine ----
// P1/P2 segment geometry for a launch of n_reads reads.
struct PartGeom {
    CountGeom geom;    // tile geometry shared by P1 and P2
    int seg_tiles;     // tiles per segment
    uint64_t nseg;     // segments (histogram columns)
    int max_win;       // windows per tile
    int scap;          // P2 staging capacity (keys)
    size_t lds_scatter;// LDS bytes of the P2 workgroup
};
PartGeom part_geometry(int L, int k, uint64_t n_reads);
// P1: hist[d * nseg + seg] = keys of segment seg with digit d = (hash >> shift) & 255
hipError_t launch_part_hist(const CountLaunch& l, const PartGeom& pg, uint64_t* hist, int shift, hipStream_t s,
                            int gbits = 0);
// key-range passes: pass histogram = groups [g0, g1) of a gbits = 4 P1 histogram; group totals
hipError_t launch_hist_group_sum(const uint64_t* h, uint64_t nseg, uint32_t g0, uint32_t g1, uint64_t* out,
                                 hipStream_t s);
hipError_t launch_hist_group_totals(const uint64_t* h, uint64_t nseg, uint32_t groups, uint64_t* tot, hipStream_t s);
// P2: scatter keys to out (SoA, out_stride) at base = exclusive scan of hist;
// also counts key 0 / holes / valid windows into l.stats
hipError_t launch_part_scatter(const CountLaunch& l, const PartGeom& pg, const uint64_t* base, uint64_t* out,
                               uint64_t out_stride, int shift, uint8_t* digs, hipStream_t s,
                               const uint64_t* base2 = nullptr, uint64_t* out2 = nullptr,
                               uint64_t out2_stride = 0, uint8_t* digs2 = nullptr, uint32_t fmid = 256,
                               bool aos = false);
// P3 (regional scatter, see kc_kernels.hip): rstart[257] region bounds,
// tpre[257] tile prefix per region (tiles of p3_tile(W) keys); hist holds
// 256 * ntiles u64, tmp scan_tmp_elems(256 * ntiles) u64.
int p3_tile(int W);
// digs: the P3 digit of every key (written by P2), one byte per key; pos:
// 256 * ntiles u64 (tile-major run starts); tmp: p3_tmp_elems(ntiles) u64
hipError_t launch_p3_hist(int W, const uint8_t* digs, const uint64_t* rstart, const uint64_t* tpre, uint64_t ntiles,
                          uint64_t* pos, uint64_t* tmp, int grid, hipStream_t s);
uint64_t p3_tmp_elems(uint64_t ntiles);
hipError_t launch_p3_scatter(int W, const uint64_t* kin, uint64_t* kout, uint64_t stride, const uint64_t* rstart,
                             const uint64_t* tpre, uint64_t ntiles, const uint64_t* hist, int grid, hipStream_t s);
// P4: starts[b] for b in [0, 2^bits]: first key index of bucket b (= hash >> (64 - bits))
hipError_t launch_bucket_bounds(int W, const uint64_t* keys, uint64_t stride, uint64_t n, int bits, uint64_t* starts,
                                hipStream_t s);
// P5: LDS counting per bucket -> records (SoA, rec_cap stride) at *rec_cursor;
// LDS overflow -> global table -> spill (SoA, spill_cap stride) counted in
// stats[ST_SPILL2_FILL]
int bucket_lds_slots(int W);
hipError_t launch_count_buckets(int W, const uint64_t* keys, uint64_t stride, const uint64_t* starts,
                                uint32_t nbuckets, uint64_t* rec_keys, uint32_t* rec_cnts, uint64_t rec_cap,
                                uint64_t* rec_cursor, uint64_t* table, uint64_t cap, uint64_t* spill,
                                uint64_t spill_cap, uint64_t* stats, uint32_t probe_limit, uint32_t lcap, int grid,
                                uint64_t* desc_key, uint64_t* desc_start, uint32_t* desc_len, uint64_t desc_cap,
                                hipStream_t s, bool distinct = false, const uint64_t* sub_starts = nullptr,
                                const uint8_t* run_flags = nullptr, const uint8_t* bucket_flags = nullptr,
                                uint32_t run_per = 0);
// P5s (pre-split buckets): runs of sub-buckets of at most sort_runs_keys(W)
// keys sorted in LDS into key-ordered record segments (descriptor bit 31 set);
// runs it cannot take are flagged (run_flags[b * 256 + s0], bucket_flags[b],
// *nflag) for launch_count_buckets with the same flags and run_per.
int sort_runs_keys(int W);
hipError_t launch_sort_runs(int W, const uint64_t* keys, uint64_t stride, const uint64_t* sub_starts,
                            uint32_t nbuckets, uint64_t* rec_keys, uint32_t* rec_cnts, uint64_t rec_cap,
                            uint64_t* rec_cursor, uint64_t* stats, uint64_t* desc_key, uint64_t* desc_start,
                            uint32_t* desc_len, uint64_t desc_cap, uint8_t* run_flags, uint8_t* bucket_flags,
                            uint32_t* nflag, int grid, hipStream_t s, void* packed = nullptr,
                            uint64_t pk_base = 0);
// Direct mode (packed != nullptr): records go to packed + (pk_base + run's first
// key + rank) records of 2W+1 u32; *rec_cursor counts them (fewer than the keys
// when runs held equal keys: then launch_packed_seg_copy closes the gaps).
hipError_t launch_packed_seg_copy(int W, const void* src, void* dst, const uint32_t* order, const uint64_t* dstart,
                                  const uint32_t* dlen, const uint64_t* out_off, uint64_t ndesc, uint64_t base,
                                  int grid, hipStream_t s);
// Starts of the 256 sub-buckets per region after a regional radix pass by key
// bits 40..47 (rp_hist/rp_scatter over nreg regions): nreg * 256 + 1 entries
hipError_t launch_sub_starts(const uint64_t* rstart, const uint64_t* tpre, const uint64_t* pos, uint32_t nreg,
                             uint64_t n, uint64_t* sub, hipStream_t s);
// Finish without a global sort (see kc_kernels.hip): lens_sorted[i] = len[order[i]];
// seg_sort writes each descriptor's records sorted at out_off[i].
hipError_t launch_desc_prep(const uint32_t* order, const uint32_t* len, uint64_t n, uint64_t* lens_sorted,
                            hipStream_t s);
size_t seg_sort_lds(int W);
hipError_t launch_iota_u32(uint32_t* out, uint64_t n, hipStream_t s);
// out[i] = (keys[i] >> shift) & 255 for i in [lo, hi) (word 0 of SoA records)
hipError_t launch_key_digits(const uint64_t* keys, uint64_t lo, uint64_t hi, int shift, uint8_t* out, hipStream_t s);
// *out = base[n - 1] + counts[n - 1] (an exclusive scan's total), n >= 1
hipError_t launch_sum_last(const uint64_t* base, const uint64_t* counts, uint64_t n, uint64_t* out, hipStream_t s);
// seg_sort descriptors of ng groups from their bounds starts[0..ng]: order =
// identity, len = length | tag << 24; *longest (zeroed by the caller) = the
// longest group
hipError_t launch_group_desc(const uint64_t* starts, uint64_t ng, uint32_t tag, uint32_t* order, uint32_t* len,
                             uint64_t* longest, hipStream_t s);
// fb: ndesc u32 + fb_n: 1 u64 of scratch (the LSD fallback list). With
// `packed`, records go straight to SortedKMerFile layout there (okeys/ocnts
// unused).
hipError_t launch_seg_sort(int W, const uint64_t* rkeys, const uint32_t* rcnts, uint64_t rstride, const uint32_t* order,
                           const uint64_t* dstart, const uint32_t* dlen, const uint64_t* out_off, uint64_t ndesc,
                           uint64_t* okeys, uint32_t* ocnts, uint64_t ostride, uint64_t* stats, uint32_t* fb,
                           uint64_t* fb_n, int grid, hipStream_t s, void* packed,
                           const uint64_t* dkey = nullptr);
// segmented sum of sorted records (out_cnts zeroed by the caller)
hipError_t launch_reduce_add(int W, const uint64_t* keys, uint64_t stride, const uint32_t* cnts, uint64_t n,
                             const uint32_t* flags, const uint32_t* pos, uint64_t* out_keys, uint64_t ostride,
                             uint32_t* out_cnts, hipStream_t s);

// Table -> dense SoA (keys W x out_cap words, counts) in slot order; *cursor
// (device u64) receives the number of records. tmp: compact_tmp_elems() u64.
hipError_t launch_compact(int W, const uint64_t* table, uint64_t cap, uint64_t* keys, uint32_t* cnts,
                          uint64_t out_cap, uint64_t* cursor, uint64_t* tmp, hipStream_t s);
uint64_t compact_tmp_elems();
// Appends (0^W, stats[ST_KEY0]) at index *cursor when stats[ST_KEY0_PRESENT].
hipError_t launch_append_key0(int W, uint64_t* keys, uint32_t* cnts, uint64_t out_cap, uint64_t* cursor,
                              const uint64_t* stats, hipStream_t s);

// OR / AND of every key word (2*W u64 at `bits`: or[0..W), and[W..2W)); host
// must pre-set or = 0, and = ~0.
hipError_t launch_key_bits(int W, const uint64_t* keys, uint64_t stride, uint64_t n, uint64_t* bits, hipStream_t s);

// One LSD pass on digit (word, shift) of SoA records: keys (W arrays at
// `stride`), optional vals. hist must hold sort_hist_elems(grid) u64.
int sort_grid(uint64_t n);
uint64_t sort_hist_elems(int grid);
// hashed: the digit is taken from the key hash instead of key word `word`.
hipError_t launch_sort_pass(int W, const uint64_t* keys_in, uint64_t* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, uint64_t stride, uint64_t n, int word, int shift, uint64_t* hist,
                            int grid, bool hashed, hipStream_t s);

// Exclusive scan of n elements (device-wide); tmp must hold scan_tmp_elems(n).
uint64_t scan_tmp_elems(uint64_t n);
hipError_t launch_scan_u32(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* tmp, hipStream_t s);
hipError_t launch_scan_u64(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* tmp, hipStream_t s);

// Run-length reduce of sorted keys (counts = run lengths).
hipError_t launch_rle_heads(int W, const uint64_t* keys, uint64_t stride, uint64_t n, uint32_t* flags,
                            hipStream_t s);
hipError_t launch_rle_scatter(int W, const uint64_t* keys, uint64_t stride, uint64_t n, const uint32_t* flags,
                              const uint32_t* pos, uint64_t* out_keys, uint64_t out_stride, uint32_t* head_idx,
                              hipStream_t s);
hipError_t launch_rle_counts(const uint32_t* head_idx, uint64_t m, uint64_t n, uint32_t* cnts, hipStream_t s);

// SoA -> SortedKMerFile bytes (rs = 8W+4 per record).
hipError_t launch_pack(int W, const uint64_t* keys, uint64_t stride, const uint32_t* cnts, uint64_t n, void* out,
                       hipStream_t s);

// Key-space partition: bounds[o] = first packed record with owner >= o
// (o in [0, world]); unpack packed records into SoA.
hipError_t launch_owner_bounds(const void* packed, int rs, uint64_t n, uint32_t world, uint64_t* bounds,
                               hipStream_t s);
// Merge path of two sorted SoA runs (A first on equal keys) into ko/co
// (stride so); split: merge_split_elems(na + nb) u64 scratch.
hipError_t launch_merge(int W, const uint64_t* ka, const uint32_t* ca, uint64_t sa, uint64_t na, const uint64_t* kb,
                        const uint32_t* cb, uint64_t sb, uint64_t nb, uint64_t* ko, uint32_t* co, uint64_t so,
                        uint64_t* split, hipStream_t s);
uint64_t merge_split_elems(uint64_t n);
// Merge path over two sorted, deduplicated packed runs (SortedKMerFile
// records) into `out` (packed, sorted; a key of both runs leaves two adjacent
// records and sets *dup). split: merge_packed_split_elems(W, na + nb) u64.
hipError_t launch_merge_packed(int W, const void* a, uint64_t na, const void* b, uint64_t nb, void* out,
                               uint64_t* split, uint32_t* dup, hipStream_t s);
uint64_t merge_packed_split_elems(int W, uint64_t n);
hipError_t launch_unpack(int W, const void* packed, uint64_t n, uint64_t* keys, uint64_t stride, uint32_t* cnts,
                         hipStream_t s);

// FASTQ block index (K1).
uint64_t fq_chunks(const void* base, uint64_t n);
hipError_t launch_fq_count(const uint8_t* base, uint64_t n, uint64_t* counts, hipStream_t s);
hipError_t launch_fq_emit(const uint8_t* base, uint64_t n, const uint64_t* line_base, uint64_t* seq_off,
                          uint64_t* seq_end, uint64_t max_rec, uint64_t* stats, hipStream_t s);
hipError_t launch_fq_validate(const uint64_t* seq_off, const uint64_t* seq_end, uint64_t n_rec, int L,
                              uint64_t* stats, hipStream_t s,
                              bool at_most = false);
// K1 emit + E in one pass (after fq_count + scan): codes / inval of every read
// of the block (groups_per_read(L) each, read r at r * G), the same format
// checks as fq_emit + fq_validate; seq_off / seq_end are not written.
hipError_t launch_fq_encode(const uint8_t* base, uint64_t n, const uint64_t* line_base, uint64_t max_rec, int L,
                            uint32_t* codes, uint16_t* inval, uint64_t* stats, hipStream_t s);
// The same for variable-length reads (KC_FLAG_VARLEN): sequences of 0..L
// bases encoded as launch_encode_reads_var does (slot padding, rlen, ST_VHOLE,
// ST_VWIN); ERR_FQ_LIST when a half holds more records than its list (then
// index the block with the two-pass path).
// The fused variable-length index + encode handles reads up to ~4060 bases (else two-pass)
bool fq_encode_var_ok(int L);
// One-pass FASTQ index + encode (fixed L, fq_spec_ok(L)): chunk c's records at
// rows [c R, c R + R), R = fq_spec_rows_per_chunk(L), rows past them empty
// (rlen 0, every base not-ACGT); cnt[c] = the chunk's newlines, phase[c] = its
// guessed line phase | 4 when not found. Then scan cnt into line bases and run
// launch_fq_spec_verify, which sets ERR_FQ_SPEC in stats[ST_ERR] on a miss.
bool fq_spec_ok(int L);
uint64_t fq_spec_rows_per_chunk(int L);
hipError_t launch_fq_encode_spec(const uint8_t* base, uint64_t n, int L, uint32_t* codes, uint16_t* inval,
                                 uint16_t* rlen, uint64_t* cnt, uint8_t* phase, uint64_t* stats, hipStream_t s);
hipError_t launch_fq_spec_verify(const uint64_t* line_base, const uint8_t* phase, uint64_t nch, uint64_t* stats,
                                 hipStream_t s);
hipError_t launch_fq_encode_var(const uint8_t* base, uint64_t n, const uint64_t* line_base, uint64_t max_rec, int L,
                                int k, uint32_t* codes, uint16_t* inval, uint16_t* rlen, uint64_t* stats,
                                hipStream_t s);

// ---- super-k-mer engine (kc_skm.inl) ----
struct SkmGeom {
    bool ok;        // (L, k) supported: W <= 3, k >= 18, L - k + 1 <= 4096
    int m;          // minimizer length
    int Kp;         // key span in bases (k, or 32W when the last word is not masked)
    int nmax;       // keys per record at most
    int R, NG, HS;  // F tile: reads, code groups per read, m-mer hash slots per read
    int hq;         // F: m-mer positions per hash item
    size_t lds;     // F dynamic LDS bytes
};
SkmGeom skm_geometry(int L, int k);
bool skm_f3_applies(int L, int k);  // the F3 front end counts (L, k) batches
// F: records (RW = W + 1 words, SoA at pool_cap) of the launch's reads; *pool_cursor
// (zeroed by the caller) ends as the number of records handed out (padding
// included); > pool_cap means the pool overflowed and nothing may be used.
// dig1 (optional, pool_cap bytes): each record's low bucket byte, the first
// grouping pass's digit (its histogram then reads a byte per record, not word 0)
hipError_t launch_skm_front(const CountLaunch& l, const SkmGeom& g, uint64_t* pool, uint64_t pool_cap,
                            uint64_t* pool_cursor, int grid_cap, hipStream_t s, uint8_t* dig1 = nullptr);
// rp_*: radix grouping passes over NW-word SoA items (+ optional u32 payload)
int rp_tile(int NW, bool pay);
uint64_t* rp_digit_base(uint64_t* tmp, uint64_t ntiles);  // exclusive digit bases after launch_rp_hist
// digit = digs[i] (digs != nullptr) or (w0[i] >> shift) & 255; tmp: p3_tmp_elems(ntiles); pos: 256 * ntiles
hipError_t launch_rp_hist(const uint8_t* digs, const uint64_t* w0, int shift, const uint64_t* rstart,
                          const uint64_t* tpre, int nreg, uint64_t ntiles, uint32_t tile, uint64_t* pos,
                          uint64_t* tmp, int grid, hipStream_t s);
// MSD regional histogram: digit (w0[i] >> shift) & 255, runs placed inside
// their region (regions stay in order, each sorted by the digit); cnt_t:
// 256 * ntiles u32 scratch, pos: 256 * ntiles run starts
hipError_t launch_rp_hist_regional(const uint64_t* w0, int shift, const uint64_t* rstart, const uint64_t* tpre,
                                   int nreg, uint64_t ntiles, uint32_t tile, uint64_t* pos, uint32_t* cnt_t, int grid,
                                   hipStream_t s, const uint8_t* digs = nullptr);
// istride / ostride 0: the input / output items are NW consecutive words each
// (AoS, as P2 writes them and P3b reads P3's output), else NW word arrays
hipError_t launch_rp_scatter(int NW, bool pay, const uint64_t* kin, uint64_t istride, uint64_t* kout,
                             uint64_t ostride, const uint32_t* pin, uint32_t* pout, const uint64_t* rstart,
                             const uint64_t* tpre, int nreg, uint64_t ntiles, const uint64_t* pos, int dshift,
                             uint8_t* emit, int eshift, int grid, hipStream_t s);
int skm_lds_slots(int W);
int seg_sort_cap(int W);  // longest segment seg_sort_k takes
// P5a (W = 1): per bucket b of [b0, b1), its distinct records written back in
// place at the front of its range of recs (2 x stride SoA), their
// multiplicities at the same indices of cnt; dlen[b] = their number
// (kRawList 0xffffffff: the table filled, records left as they were)
// A bucket whose distinct records overflow the LDS table is deduplicated
// again in hash-split passes into a list reserved from *over_cursor (records
// of recs / cnt below over_limit, free), dpos[b] its start, dlen[b] =
// 0x80000000 | its length; no room or no over_cursor: left raw.
hipError_t launch_count_rec(uint64_t* recs, uint64_t stride, const uint64_t* starts, uint32_t b0, uint32_t b1,
                            uint32_t* cnt, uint32_t* dlen, int grid, hipStream_t s, uint64_t* over_cursor = nullptr,
                            uint64_t over_limit = 0, uint64_t* dpos = nullptr);
// stats[ST_DEDUP] += sum over buckets [0, nb) of dlen[b] (raw: the bucket's records)
hipError_t launch_dedup_total(const uint32_t* dlen, const uint64_t* starts, uint32_t nb, uint64_t* stats,
                              hipStream_t s);
struct SkmDedup {
    const uint32_t* cnt;  // P5a output
    const uint32_t* len;
    const uint64_t* pos;  // overflow lists' starts (len flag 0x80000000)
};
// buckets [b0, b1); count_keys: add the buckets' key counts to stats[ST_P5_KEYS];
// dd (optional): P5a's lists, walked instead of the buckets' records
hipError_t launch_count_skm(int W, int k, const uint64_t* recs, uint64_t stride, const uint64_t* starts,
                            uint32_t b0, uint32_t b1, bool count_keys, uint64_t* rec_keys, uint32_t* rec_cnts, uint64_t rec_cap,
                            uint64_t* rec_cursor, uint64_t* table, uint64_t cap, uint64_t* spill, uint64_t spill_cap,
                            uint64_t* stats, uint32_t probe_limit, uint32_t lcap, int grid, hipStream_t s,
                            const SkmDedup* dd = nullptr, uint8_t* rec_dig = nullptr);

// Synthetic FASTQ generator (bench/test input).
struct SynthArgs {
    uint64_t first, n, seed, genome, n_threshold;
    int64_t L;
    int64_t Lmin = 0;  // variable read lengths in [Lmin, L] (0: fixed)
    int layout = 0;    // 1: concatenated sequences (reference chunk layout)
};
// Coverage sketch of encoded reads (kc_kernels.hip sketch_k): fingerprints of
// the group-aligned k-mers whose hash has rate_bits low zero bits (a 2^-rate
// sample by k-mer, so every copy of a sampled k-mer is kept) appended to out
// (cap), count in *counter
hipError_t launch_sketch(const uint32_t* codes, const uint16_t* inval, uint64_t n_reads, int L, int k, int rate_bits,
                         uint64_t* out, uint64_t cap, uint64_t* counter, hipStream_t s);
// Distinct fingerprints among the first min(*counter, cap) of fp, counted by
// inserting them into `set` (2^set_bits zeroed u64 slots, cap <= half of them);
// the count is added to *distinct
hipError_t launch_sketch_distinct(const uint64_t* fp, const uint64_t* counter, uint64_t cap, uint64_t* set,
                                  int set_bits, uint64_t* distinct, hipStream_t s);
hipError_t launch_synth(const SynthArgs& a, char* out, hipStream_t s);
void synth_host(const SynthArgs& a, char* out);
uint64_t synth_bytes(uint64_t first, uint64_t n, int64_t L, int layout);

}  // namespace kc
