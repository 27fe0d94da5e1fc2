// kc_kernels.hip — hand-written CDNA4 (gfx950, wave64) kernels of the k-mer
// count path. Design and rooflines: DESIGN.md. Reference semantics restated
// here:
//   bitEncode     GPUHandler.cu:10-111  -> count_kmers stage 2 (LDS encode)
//   extractKMers  GPUHandler.cu:129-233 -> count_kmers stage 3 (window keys)
//   TBB hash      KMerCounter.cpp:61-82 -> count_kmers stage 3 (HBM table insert)
//   sortKmers     GPUHandler.cu:300-327 -> sort_* (LSD radix, disabled in the ref)
//   reduceKMers   GPUHandler.cu:329-360 -> rle_* (run-length reduce of spill runs)
//   readData      FASTQFileReader.cpp:49-89 -> fq_* (FASTQ block index)
#include <hip/hip_runtime.h>

#include "kc_device.h"
#include <cstdlib>
#include <type_traits>
#include "kc_synth.h"

namespace kc {

typedef uint64_t u64;
typedef unsigned int u32;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
// a volatile 16-byte LDS load (ds_read_b128): the cast pins the LDS address
// space, which a generic volatile pointer loses (it would become a FLAT load)
typedef __attribute__((address_space(3))) volatile v2u64 lds_v2u64;

// key i of a key array into k: W word arrays at `stride`, or (stride 0) W
// consecutive words per key (AoS; one 16-byte load at W = 2)
template <int W>
__device__ __forceinline__ void load_key(const u64* __restrict__ keys, u64 stride, u64 i, u64 (&k)[W]) {
    if (stride == 0) {
        if constexpr (W == 2) {
            const v2u64 v = *(const v2u64*)(keys + 2 * i);
            k[0] = v.x;
            k[1] = v.y;
        } else {
#pragma unroll
            for (int j = 0; j < W; j++) k[j] = keys[i * W + j];
        }
    } else {
#pragma unroll
        for (int j = 0; j < W; j++) k[j] = keys[(u64)j * stride + i];
    }
}

constexpr int kBlock = 256;  // 4 waves of 64
constexpr int kWave = 64;

static inline u64 hmin(u64 a, u64 b) { return a < b ? a : b; }

// ---------------------------------------------------------------------------
// wave helpers (wave64)
// ---------------------------------------------------------------------------

__device__ __forceinline__ u32 lane_id() { return __lane_id(); }

__device__ __forceinline__ u64 lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Block-uniform values read from LDS, made scalar so the branches (and the
// barriers under them) are uniform to the compiler as well.
__device__ __forceinline__ u32 uni32(u32 v) { return __builtin_amdgcn_readfirstlane(v); }
// v <= lim for a 64-bit uniform v as two 32-bit compares: hipcc (ROCm 7.2)
// lowers a uniform 64-bit unsigned compare to a VALU compare in VCC and can
// then select on SCC (a stale carry) — seen in sort_runs_k's run length
__device__ __forceinline__ bool le64_32(u64 v, u32 lim) { return (u32)(v >> 32) == 0u && (u32)v <= lim; }
__device__ __forceinline__ u64 uni64(u64 v) {
    return ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(v >> 32)) << 32) |
           (u64)(u32)__builtin_amdgcn_readfirstlane((u32)v);
}


// Wave-aggregated atomicAdd of `mine` (per lane) to *ctr; returns this lane's
// exclusive position (ctr_old + prefix of lower active lanes).
__device__ __forceinline__ u64 wave_reserve(u64* ctr, bool want) {
    u64 m = __ballot(want);
    u64 base = 0;
    if (m) {
        int leader = __ffsll((long long)m) - 1;
        if ((int)lane_id() == leader) base = atomicAdd((unsigned long long*)ctr, (unsigned long long)__popcll(m));
        base = __shfl(base, leader);
    }
    return base + (u64)__popcll(m & lanemask_lt());
}

__device__ __forceinline__ void wave_add(u64* ctr, u64 v) {
    // reduce v over the active lanes, one atomic per wave
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    u64 act = __ballot(1);
    if ((int)lane_id() == __ffsll((long long)act) - 1 && v) atomicAdd((unsigned long long*)ctr, v);
}

// n / d for n, d < 2^16 with one mul_hi (m = ceil(2^32 / d) is exact there)
struct FastDivU {
    u32 d, m;
    __device__ __forceinline__ explicit FastDivU(u32 dd) : d(dd), m((u32)((0x100000000ull + dd - 1) / dd)) {}
    __device__ __forceinline__ u32 div(u32 v) const { return d == 1 ? v : __umulhi(v, m); }
};

__device__ __forceinline__ u64 mix64(u64 x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <int W>
__device__ __forceinline__ u64 hash_key(const u64 (&key)[W]) {
    u64 h = mix64(key[0] ^ 0x9e3779b97f4a7c15ull);
#pragma unroll
    for (int j = 1; j < W; j++) h = mix64(h ^ key[j]);
    return h;
}

// Block-wide exclusive scan of one u32 per thread (256 threads). `lds` holds
// >= 4 u32. Returns the exclusive prefix; *total receives the block sum.
__device__ __forceinline__ u32 block_excl_scan(u32 v, u32* lds, u32* total) {
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u32 x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        u32 y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wave] = x;
    __syncthreads();
    u32 w0 = lds[0], w1 = lds[1], w2 = lds[2], w3 = lds[3];
    u32 before = (wave > 0 ? w0 : 0) + (wave > 1 ? w1 : 0) + (wave > 2 ? w2 : 0);
    *total = w0 + w1 + w2 + w3;
    __syncthreads();
    return before + x - v;
}

// ---------------------------------------------------------------------------
// K2: count_kmers<W> — fused FASTQ/chunk tile stage -> 2-bit encode -> window
// keys -> open-addressed HBM table insert (CAS claim + atomic count).
//
// One workgroup (256 threads) per tile of R reads:
//   1. stage: the 16-byte-aligned span of every read is copied into LDS with
//      coalesced 16 B loads (one read per aligned run of lanes);
//   2. encode: each (read, 16-base group) -> a u32 of 2-bit codes
//      (A0 C1 G2 T3, other bytes 3, MSB-first as bitEncode) and a 16-bit
//      not-ACGT mask (bitEncode's filter); groups past L are zero, which is
//      the reference's zero padding of the last word / past-end reads;
//   3. windows: lane -> window (r, p); the W key words are funnel-shifted out
//      of three consecutive code groups (extractKMers' shift-combine), the last
//      word masked to k%32 bases only when ceil(k/4) < 8W (GPUHandler.cu:181);
//      valid windows (no masked base in p..p+k-1) are inserted into the table.
// Key 0^W never enters the table (0 is the EMPTY key): it is counted with one
// wave-aggregated atomic into stats[ST_KEY0]. Any invalid window sets
// stats[ST_KEY0_PRESENT] (the zeroed hole record of extractKMers reaches the
// host hash as key 0, count 0: GPUHandler.cu:466 -> KMerCounter.cpp:70).
// Inserts that exceed probe_limit go to the spill buffer (sorted into runs and
// merged later), so no key is ever lost.
// ---------------------------------------------------------------------------

struct CountArgs {
    const uint8_t* base;
    const u64* seq_off;
    u64 read0, n_reads;
    int L, k, R, NG, raw_stride;
    u64* table;
    u64 cap;
    u64* spill;
    u64 spill_cap;
    u64* stats;
    u32 probe_limit;
    const unsigned short* rlen;  // CODES: a row of length 0 (one-pass empty row) is no read
};

// Reads per tile that keep the kRoll-window chunks of a tile close to a whole
// number of 256-lane rounds (R_max bounds R).
static int balance_reads(int R_max, int nw, int nt = kBlock) {
    const int nchr = (nw + 7) / 8;
    int best = R_max;
    double best_eff = 0;
    for (int R = R_max; R >= 1 && R >= R_max / 2; R--) {
        int ch = R * nchr;
        int rounds = (ch + nt - 1) / nt;
        double eff = (double)ch / (rounds * nt);
        if (eff > best_eff + 1e-9) {
            best_eff = eff;
            best = R;
        }
    }
    return best;
}

CountGeom count_geometry(int L, int k) {
    CountGeom g;
    int W = (k + 31) / 32;
    int nw = L - k + 1;
    g.NG = (L + 15) / 16 + 2 * W + 3;
    g.raw_stride = ((L + 31 + 15) / 16) * 16 + 16;
    // aim for ~8 window runs per thread, bounded by a 48 KiB LDS budget
    int R = (64 * kBlock + nw - 1) / (nw > 0 ? nw : 1);
    if (R < 1) R = 1;
    if (R > 64) R = 64;
    auto bytes = [&](int r) {
        return (size_t)r * g.raw_stride + (size_t)r * g.NG * 8 + (size_t)r * 8 + 16;
    };
    while (R > 1 && bytes(R) > 48 * 1024) R--;
    R = balance_reads(R, nw);
    g.R = R;
    g.lds = (bytes(R) + 15) & ~(size_t)15;
    return g;
}

// W == 1: slot = {key, count}. Returns true when counted; *claimed when this
// insert took an empty slot. A key word only ever changes 0 -> key, so a plain
// (possibly stale) load can only be wrong in the EMPTY direction: a non-zero
// value is the slot's final key and a repeat costs one atomic (the count add);
// an EMPTY reading is confirmed or corrected by the CAS.
// w: the count added (a deduplicated super-k-mer's multiplicity; 1 otherwise)
__device__ __forceinline__ bool insert_w1(u64 key, u64* __restrict__ table, u64 cap, u32 limit, bool* claimed,
                                          u32 w = 1u) {
    u64 s = __umul64hi(mix64(key ^ 0x9e3779b97f4a7c15ull), cap);
    for (u32 pr = 0; pr < limit; ++pr) {
        u64* slot = table + 2 * s;
        u64 cur = __builtin_nontemporal_load(slot);
        if (cur == 0ull) cur = atomicCAS((unsigned long long*)slot, 0ull, (unsigned long long)key);
        if (cur == 0ull || cur == key) {
            atomicAdd((unsigned int*)(slot + 1), w);
            *claimed = (cur == 0ull);
            return true;
        }
        if (++s == cap) s = 0;
    }
    return false;
}

// W >= 2: slot = {key[W], count:u32, state:u32}; state 0 EMPTY, 1 WRITING,
// 2 READY. The claimer writes the key words with agent-scope (sc1,
// write-through) stores, drains them, then publishes state 2; readers poll the
// state and read the words with sc1 loads (MI355X_MICROARCH.md "Valid forms").
// A writer that does not publish within the spin bound makes the key spill,
// which keeps the count exact.
template <int W>
__device__ __forceinline__ bool insert_wide(const u64 (&key)[W], u64* __restrict__ table, u64 cap, u32 limit,
                                            bool* claimed, u32 w = 1u) {
    // One attempt per iteration and no spin inside divergent code: a lane that
    // finds the slot being published (state 1) retries it next iteration. The
    // claimer publishes within its own iteration, so a lane of the same
    // wavefront can never wait on a masked-off claimer.
    constexpr int SW = (W <= 3) ? 4 : 8;
    u64 s = __umul64hi(hash_key<W>(key), cap);
    u32 pr = 0, waits = 0;
    for (;;) {
        u64* slot = table + SW * s;
        u32* cnt = (u32*)(slot + W);
        u32* state = cnt + 1;
        u32 st = __hip_atomic_load(state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (st == 0u) {
            u32 prev = atomicCAS(state, 0u, 1u);
            if (prev == 0u) {
#pragma unroll
                for (int j = 0; j < W; j++)
                    __hip_atomic_store(slot + j, key[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicAdd(cnt, w);
                __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(state, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *claimed = true;
                return true;
            }
            st = prev;
        }
        if (st == 1u) {
            if (++waits > (1u << 22)) return false;  // claimer lost: treat as a full probe
            continue;
        }
        bool eq = true;
#pragma unroll
        for (int j = 0; j < W; j++)
            eq = eq && (__hip_atomic_load(slot + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == key[j]);
        if (eq) {
            atomicAdd(cnt, w);
            return true;
        }
        if (++pr >= limit) return false;
        if (++s == cap) s = 0;
    }
}

__device__ __forceinline__ u32 bytes_to_codes(u32 word, int nvalid, u32* bad_bits) {
    // 4 bytes of text -> 4 2-bit codes in the low byte (first byte highest) and
    // a 4-bit not-ACGT mask (first byte highest); bytes >= nvalid are zero.
    u32 codes = 0, bad = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        u32 c = (word >> (8 * b)) & 0xffu;
        u32 ok = (c == 'A') | (c == 'C') | (c == 'G') | (c == 'T');
        u32 code = ok ? (((c >> 2) ^ (c >> 1)) & 3u) : 3u;
        if (b >= nvalid) {
            code = 0;
            ok = 1;
        }
        codes |= code << (6 - 2 * b);
        bad |= (ok ^ 1u) << (3 - b);
    }
    *bad_bits = bad;
    return codes;
}

// Sinks of the count front end (stages 1-3 above are shared):
//   SINK_TABLE   : insert into the global open-addressed table (engine "table")
//   SINK_HIST    : per-segment histogram of the partition digit (engine
//                  "partition", pass P1); no statistics are touched
//   SINK_SCATTER : per-tile LDS counting sort by the digit, then coalesced
//                  writes of the keys to their segment's slice of each digit's
//                  region (pass P2)
enum Sink { SINK_TABLE = 0, SINK_HIST = 1, SINK_SCATTER = 2 };

struct PartArgs {
    u64* hist;        // HIST: counts[d * nseg + seg]
    const u64* base;  // SCATTER: exclusive scan of hist (global key positions)
    u64* out;         // SCATTER: keys, SoA with out_stride
    u64 out_stride;
    u64 nseg;
    int seg_tiles;    // tiles per segment
    int shift;        // digit = (hash >> shift) & 255
    int max_win;      // windows per tile (R * windows per read)
    int scap;         // SCATTER staging capacity (keys, >= max_win)
    int skip;         // timing experiments only (KC_P2_SKIP): 1 flush writes, 2 staging, 4 whole sink
    unsigned char* digs;  // SCATTER: the P3 digit (word0 >> 56) of each written key
    const u32* codes; // CODES front end: encoded reads (kernel E), G u32 per read
    const unsigned short* inval;  //      not-ACGT masks, G u16 per read
    int G;            //                  16-base groups per read
    u32 flo, fhi;     // key-range pass: only keys with word0 >> 56 in [flo, fhi) (P1 and P2)
    int gbits;        // HIST: 2^gbits groups of word0 >> 56 (its top gbits bits), 256 digits each
    // SCATTER, two key-range passes in one walk: keys with word0 >> 56 in
    // [fmid, fhi) go to out2 (stride out2_stride, digit bytes digs2, run
    // starts base2) as the second pass's P2 output
    u64* out2;
    u64 out2_stride;
    const u64* base2;
    unsigned char* digs2;
    u32 fmid;
    int no_stats;     // key-range pass after the first: valid / key-0 statistics not counted again
    int aos;          // SCATTER: keys written as W consecutive words (16-byte stores at W = 2), not SoA
};

static size_t sink_lds_host(int W, int sink, int scap) {
    if (sink == SINK_HIST) return 256 * 4;
    if (sink == SINK_SCATTER)
        return 2 * 512 * 8 + 516 * 4 + 512 * 4 + 64 + (size_t)W * 8 * (scap + 1) + 2 * (size_t)scap + 16;
    return 0;
}

constexpr int kRoll = 8;  // consecutive windows per lane

// 32 bases starting at base index b of a read's LDS code groups (16 bases per
// u32, first base highest), as one MSB-first word.
__device__ __forceinline__ u64 code_word(const u32* cr, int b) {
    const int g = b >> 4, o = b & 15;
    const u64 hi = ((u64)cr[g] << 32) | (u64)cr[g + 1];
    return o ? ((hi << (2 * o)) | (u64)(cr[g + 2] >> (32 - 2 * o))) : hi;
}

// Exclusive scan of NB per-digit values held by threads 0..NB-1 of a block of
// any size (waves 0..NB/64-1 scan, one barrier that every thread executes).
// scratch: >= NB/64 u32. Threads >= NB get 0.
template <int NB = 256>
__device__ __forceinline__ u32 digit_scan256(u32 v, u32* scratch, int tid) {
    const int lane = lane_id(), wave = tid >> 6;
    u32 inc = v;
    if (tid < NB) {
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        if (lane == 63) scratch[wave] = inc;
    }
    __syncthreads();
    u32 pre = 0;
    if (tid < NB)
        for (int w = 0; w < wave; w++) pre += scratch[w];
    return tid < NB ? pre + inc - v : 0u;
}

constexpr int kPrefetch = 4;  // code words prefetched per thread (CODES front end)

// NT threads per workgroup (256, or 1024 for the P2 scatter: 16 waves per CU
// with twice the staging capacity); per-digit arrays are handled by the first
// 256 threads.
template <int W, int SINK, bool CODES, int NT>
__global__ __launch_bounds__(NT) void count_front(CountArgs a, PartArgs pa) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* raw = smem;
    u32* codes = (u32*)(smem + (size_t)a.R * a.raw_stride);
    u32* inval = codes + a.R * a.NG;
    u32* lead = inval + a.R * a.NG;
    u32* rflag = lead + a.R;
    // sink region (16-byte aligned); offset arithmetic on smem keeps the LDS
    // address space (an integer round trip would turn every access into FLAT)
    const size_t sk_off = (((size_t)a.R * a.raw_stride + (size_t)2 * a.R * a.NG * 4 + (size_t)2 * a.R * 4) + 15) &
                          ~(size_t)15;
    unsigned char* sk = smem + sk_off;
    u32* s_hist = (u32*)sk;                      // HIST
    // SCATTER slots: digit d of the (first) pass at d, of the second pass at 256 + d
    u64* s_cur = (u64*)sk;                       // SCATTER: global cursor of each slot's run
    u64* s_gb = s_cur + 512;                     //          flush: s_cur[d] - start of d in flush order
    u32* s_cnt = (u32*)(s_gb + 512);             //          staged keys per slot (+ trash counter 512)
    u32* s_fill = s_cnt + 512 + 4;               //          rank cursor
    u32* s_misc = s_fill + 512;                  //          [0] staged count, [4..11] scan scratch
    u64* s_stage = (u64*)(s_misc + 16);          //          W x (scap + 1) staged keys (slot scap: trash);
                                                 //          the digit is recomputed from word 0
    unsigned short* s_perm = (unsigned short*)(s_stage + (size_t)W * (pa.scap + 1));  // scap flush order
    u32* scan_tmp = s_misc + 4;

    const int tid = threadIdx.x;
    const int L = a.L, k = a.k, NG = a.NG;
    const int nw = L - k + 1;
    const bool mask_last = ((k + 3) / 4) < 8 * W;
    const u64 last_mask = mask_last ? (~0ull << (64 - 2 * (k & 31))) : ~0ull;
    const int nch = (L + 30) / 16 + 1;  // 16 B chunks covering lead (<16) + L bytes
    const u64 ntiles = (a.n_reads + a.R - 1) / a.R;
    const u64 per_unit = (SINK == SINK_TABLE) ? 1 : (u64)pa.seg_tiles;
    const u64 nunits = (ntiles + per_unit - 1) / per_unit;

    u64 my_valid = 0;
    bool my_hole = false;

    // CODES: the next tile's code words are loaded into registers while the
    // current tile is processed (software pipelining across tiles and units)
    u32 pf_code[kPrefetch];
    u32 pf_inv[kPrefetch];
    u32 pf_len = 1;  // (row lengths: this thread's row of the next tile, with its codes)
    auto prefetch = [&](u64 tile) {
        const u64 r0 = tile * (u64)a.R;
        const int nr = (tile < ntiles) ? (int)min((u64)a.R, a.n_reads - r0) : 0;
        if (a.rlen) pf_len = tid < nr ? (u32)a.rlen[r0 + (u64)tid] : 1u;
#pragma unroll
        for (int j = 0; j < kPrefetch; j++) {
            const int it = tid + j * NT;
            const int r = it / NG, g = it - r * NG;
            u32 cw = 0, iv = 0;
            if (r < nr && g < pa.G) {
                const u64 idx = (r0 + (u64)r) * (u64)pa.G + (u64)g;
                cw = __builtin_nontemporal_load(pa.codes + idx);
                iv = __builtin_nontemporal_load(pa.inval + idx);
            }
            pf_code[j] = cw;
            pf_inv[j] = iv;
        }
    };
    if constexpr (CODES) prefetch(blockIdx.x * per_unit);

    for (u64 unit = blockIdx.x; unit < nunits; unit += gridDim.x) {
        if constexpr (SINK == SINK_HIST) {
            for (int i = tid; i < (256 << pa.gbits); i += NT) s_hist[i] = 0;
        } else if constexpr (SINK == SINK_SCATTER) {
            if (tid < 512) {
                s_cnt[tid] = 0;
                s_cur[tid] = tid < 256 ? pa.base[(u64)tid * pa.nseg + unit]
                                       : (pa.out2 ? pa.base2[(u64)(tid - 256) * pa.nseg + unit] : 0ull);
            }
            if (tid == 0) s_misc[0] = 0;
        }
        const u64 t_end = min(ntiles, (unit + 1) * per_unit);
        for (u64 tile = unit * per_unit; tile < t_end; tile++) {
            const u64 r0 = tile * (u64)a.R;
            const int nr = (int)min((u64)a.R, a.n_reads - r0);

            if constexpr (CODES) {
                // 1-2. code words of the tile (prefetched) into LDS; groups past
                //      the read end are zero (A, valid), as the encoder leaves them
#pragma unroll
                for (int j = 0; j < kPrefetch; j++) {
                    const int it = tid + j * NT;
                    if (it < nr * NG) {
                        codes[it] = pf_code[j];
                        inval[it] = pf_inv[j];
                    }
                }
                for (int it = tid + kPrefetch * NT; it < nr * NG; it += NT) {
                    const int r = it / NG, g = it - r * NG;
                    u32 cw = 0, iv = 0;
                    if (g < pa.G) {
                        const u64 idx = (r0 + (u64)r) * (u64)pa.G + (u64)g;
                        cw = pa.codes[idx];
                        iv = pa.inval[idx];
                    }
                    codes[it] = cw;
                    inval[it] = iv;
                }
                // flag 2: a row of length 0 (no read: its windows are skipped)
                if (tid < nr) rflag[tid] = (a.rlen && pf_len == 0u) ? 2u : 0u;
                __syncthreads();
                // issue the next tile's loads now; they land during this tile
                prefetch(tile + 1 < t_end ? tile + 1 : (unit + gridDim.x) * per_unit);
                for (int it = tid; it < nr * NG; it += NT)
                    if (inval[it]) atomicOr(&rflag[it / NG], 1u);
                __syncthreads();
            } else {
            // 1. stage the raw text of the tile's reads into LDS
            for (int it = tid; it < nr * nch; it += NT) {
                int r = it / nch, c = it - r * nch;
                u64 gr = a.read0 + r0 + (u64)r;
                u64 off = a.seq_off ? a.seq_off[gr] : gr * (u64)L;
                uintptr_t addr = (uintptr_t)(a.base + off);
                int ld = (int)(addr & 15);
                if (c == 0) lead[r] = (u32)ld;
                if (16 * c < ld + L) {
                    // streamed once: non-temporal, so the input stream does not
                    // evict the partially written output lines from L2
                    const v4u v = __builtin_nontemporal_load((const v4u*)((addr & ~(uintptr_t)15) + 16 * (uintptr_t)c));
                    *(v4u*)(raw + (size_t)r * a.raw_stride + 16 * c) = v;
                }
            }
            if (tid < nr) rflag[tid] = 0;
            __syncthreads();

            // 2. encode 16-base groups
            for (int it = tid; it < nr * NG; it += NT) {
                int r = it / NG, g = it - r * NG;
                int i0 = 16 * g;
                u32 cw = 0, iv = 0;
                if (i0 < L) {
                    int pos = (int)lead[r] + i0;
                    const u32* dw = (const u32*)(raw + (size_t)r * a.raw_stride) + (pos >> 2);
                    int sh = pos & 3;
                    u32 d0 = dw[0], d1 = dw[1], d2 = dw[2], d3 = dw[3], d4 = dw[4];
                    u32 x0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
                    u32 x1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
                    u32 x2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
                    u32 x3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
                    int left = L - i0;
                    u32 b0, b1, b2, b3;
                    u32 c0 = bytes_to_codes(x0, left, &b0);
                    u32 c1 = bytes_to_codes(x1, left - 4, &b1);
                    u32 c2 = bytes_to_codes(x2, left - 8, &b2);
                    u32 c3 = bytes_to_codes(x3, left - 12, &b3);
                    cw = (c0 << 24) | (c1 << 16) | (c2 << 8) | c3;
                    iv = (b0 << 12) | (b1 << 8) | (b2 << 4) | b3;
                }
                codes[it] = cw;
                inval[it] = iv;
                if (iv) atomicOr(&rflag[r], 1u);
            }
            __syncthreads();
            }

            // 3. windows -> keys -> sink. A lane takes a run of kRoll consecutive
            //    windows of one read: the first key is funnel-shifted out of the
            //    code groups (extractKMers' shift-combine), every further key
            //    shifts one base in (the base 32W past the window comes from a
            //    tail word; past the read end it is 0, as in the reference).
            const int nchr = (nw + kRoll - 1) / kRoll;
            const int total = nr * nchr;
            if constexpr (SINK == SINK_SCATTER) {
                const bool filt = pa.fhi - pa.flo < 256u || pa.out2 != nullptr;
                const u32 fmid = pa.out2 ? pa.fmid : 256u;  // first slot of the second pass: word0 >> 56 >= fmid
                // Two phases per run of kRoll windows. A: roll the windows once
                // to get the lane's live mask (valid, non-zero keys). One LDS
                // reservation per wave covers all kRoll steps: step s of the
                // wave owns [soff[s], soff[s] + popc(ballot_s)) and a lane's
                // slot in it is its rank among the step's live lanes, so
                // consecutive lanes write consecutive slots. B: roll again and
                // stage. No LDS round trip inside a step.
                for (int c = tid; c - (tid & 63) < total; c += NT) {
                    int r = c < total ? c / nchr : 0, p0 = 0;
                    const bool cact = c < total && !(rflag[r] & 2u);  // (a row of length 0: no windows)
                    u64 raw[W];
                    u64 tail = 0;
                    bool clean = true;
#pragma unroll
                    for (int j = 0; j < W; j++) raw[j] = 0;
                    if (cact) {
                        p0 = (c - r * nchr) * kRoll;
                        const u32* cr = codes + r * NG;
#pragma unroll
                        for (int j = 0; j < W; j++) raw[j] = code_word(cr, p0 + 32 * j);
                        tail = code_word(cr, p0 + 32 * W);
                        clean = rflag[r] == 0;
                    }
                    u32 livem = 0, zeros = 0, valids = 0;
                    {
                        u64 kr[W];
                        u64 tl = tail;
#pragma unroll
                        for (int j = 0; j < W; j++) kr[j] = raw[j];
#pragma unroll
                        for (int sstep = 0; sstep < kRoll; sstep++) {
                            const int p = p0 + sstep;
                            const bool active = cact && p < nw;
                            bool valid = active;
                            if (active && !clean) {
                                const u32* ir = inval + r * NG;
                                const int last = p + k - 1;
                                for (int gg = p >> 4; gg <= (last >> 4); gg++) {
                                    int lo = max(p - 16 * gg, 0), hi = min(last - 16 * gg, 15);
                                    u32 rm = (0xffffu >> lo) & (0xffffu << (15 - hi)) & 0xffffu;
                                    if (ir[gg] & rm) valid = false;
                                }
                            }
                            bool is_zero = (kr[W - 1] & last_mask) == 0ull;
#pragma unroll
                            for (int j = 0; j < W - 1; j++) is_zero = is_zero && (kr[j] == 0ull);
                            my_hole |= active && !valid;
                            valids += valid ? 1u : 0u;
                            zeros += (valid && is_zero) ? 1u : 0u;
                            const u64 w0 = W == 1 ? (kr[0] & last_mask) : kr[0];
                            const bool in = (u32)(w0 >> 56) - pa.flo < pa.fhi - pa.flo;
                            livem |= (valid && !is_zero && in ? 1u : 0u) << sstep;
#pragma unroll
                            for (int j = 0; j < W - 1; j++) kr[j] = (kr[j] << 2) | (kr[j + 1] >> 62);
                            kr[W - 1] = (kr[W - 1] << 2) | (tl >> 62);
                            tl <<= 2;
                        }
                    }
                    my_valid += valids;
                    if (!pa.no_stats && __ballot(zeros != 0u)) {
                        wave_add(&a.stats[ST_KEY0], zeros);
                        if (lane_id() == 0) atomicOr((unsigned long long*)&a.stats[ST_KEY0_PRESENT], 1ull);
                    }
                    // per-step ballots -> step offsets (scalar) -> one reservation
                    u64 bal[kRoll];
                    u32 soff[kRoll];
                    u32 wtot = 0;
#pragma unroll
                    for (int sstep = 0; sstep < kRoll; sstep++) {
                        bal[sstep] = __ballot((livem >> sstep) & 1u);
                        soff[sstep] = wtot;
                        wtot += (u32)__popcll(bal[sstep]);
                    }
                    if (wtot == 0 || (pa.skip & 6)) continue;
                    u32 wbase = 0;
                    if (lane_id() == 0) wbase = atomicAdd(&s_misc[0], wtot);
                    wbase = __builtin_amdgcn_readfirstlane(wbase);
                    const u64 lt = lanemask_lt();
                    if (filt) {
                        // key-range pass: about half the lanes hold no key of
                        // the range; only live lanes stage (no trash traffic)
#pragma unroll
                        for (int sstep = 0; sstep < kRoll; sstep++) {
                            if ((livem >> sstep) & 1u) {
                                u64 key[W];
#pragma unroll
                                for (int j = 0; j < W; j++) key[j] = raw[j];
                                key[W - 1] &= last_mask;
                                const u32 idx = wbase + soff[sstep] + (u32)__popcll(bal[sstep] & lt);
#pragma unroll
                                for (int j = 0; j < W; j++) s_stage[(size_t)j * (pa.scap + 1) + idx] = key[j];
                                atomicAdd(&s_cnt[((u32)(key[0] >> 56) >= fmid ? 256u : 0u) |
                                                 ((u32)(key[0] >> pa.shift) & 255u)],
                                          1u);
                            }
#pragma unroll
                            for (int j = 0; j < W - 1; j++) raw[j] = (raw[j] << 2) | (raw[j + 1] >> 62);
                            raw[W - 1] = (raw[W - 1] << 2) | (tail >> 62);
                            tail <<= 2;
                        }
                        continue;
                    }
#pragma unroll
                    for (int sstep = 0; sstep < kRoll; sstep++) {
                        // branch-free: a lane without a live key writes the trash
                        // slot scap and bumps the trash counter 256 (no exec-mask
                        // juggling on the scalar unit)
                        const bool lv = (livem >> sstep) & 1u;
                        u64 key[W];
#pragma unroll
                        for (int j = 0; j < W; j++) key[j] = raw[j];
                        key[W - 1] &= last_mask;
                        const u32 idx = lv ? wbase + soff[sstep] + (u32)__popcll(bal[sstep] & lt) : (u32)pa.scap;
                        const u32 d = (u32)(key[0] >> pa.shift) & 255u;
#pragma unroll
                        for (int j = 0; j < W; j++) s_stage[(size_t)j * (pa.scap + 1) + idx] = key[j];
                        atomicAdd(&s_cnt[lv ? d : 512u], 1u);
#pragma unroll
                        for (int j = 0; j < W - 1; j++) raw[j] = (raw[j] << 2) | (raw[j + 1] >> 62);
                        raw[W - 1] = (raw[W - 1] << 2) | (tail >> 62);
                        tail <<= 2;
                    }
                }
            } else {
                for (int c = tid; c - (tid & 63) < total; c += NT) {
                    // the loop bound is wave-uniform so every lane reaches the ballots
                    int r = c < total ? c / nchr : 0, p0 = 0;
                    const bool cact = c < total && !(rflag[r] & 2u);  // (a row of length 0: no windows)
                    u64 raw[W];
                    u64 tail = 0;
                    bool clean = true;
    #pragma unroll
                    for (int j = 0; j < W; j++) raw[j] = 0;
                    if (cact) {
                        p0 = (c - r * nchr) * kRoll;
                        const u32* cr = codes + r * NG;
    #pragma unroll
                        for (int j = 0; j < W; j++) raw[j] = code_word(cr, p0 + 32 * j);
                        tail = code_word(cr, p0 + 32 * W);
                        clean = rflag[r] == 0;
                    }
    #pragma unroll 1
                    for (int sstep = 0; sstep < kRoll; sstep++) {
                        const int p = p0 + sstep;
                        const bool active = cact && p < nw;
                        u64 key[W];
    #pragma unroll
                        for (int j = 0; j < W; j++) key[j] = active ? raw[j] : 0ull;
                        key[W - 1] &= last_mask;
                        bool valid = active;
                        if (active && !clean) {
                            const u32* ir = inval + r * NG;
                            const int last = p + k - 1;
                            for (int gg = p >> 4; gg <= (last >> 4); gg++) {
                                int lo = max(p - 16 * gg, 0), hi = min(last - 16 * gg, 15);
                                u32 rm = (0xffffu >> lo) & (0xffffu << (15 - hi)) & 0xffffu;
                                if (ir[gg] & rm) valid = false;
                            }
                        }
                        my_hole |= active && !valid;
                        bool is_zero = true;
        #pragma unroll
                        for (int j = 0; j < W; j++) is_zero = is_zero && (key[j] == 0ull);
                        const bool live = valid && !is_zero;

                        if constexpr (SINK == SINK_HIST) {
                            const u32 top = (u32)(key[0] >> 56);
                            if (live && top - pa.flo < pa.fhi - pa.flo)
                                atomicAdd(&s_hist[((top >> (8 - pa.gbits)) << 8) | ((u32)(key[0] >> pa.shift) & 255u)], 1u);
                        } else {
                            // key 0^W: one atomic per wave
                            u64 zmask = __ballot(valid && is_zero);
                            if (zmask) {
                                if ((int)lane_id() == __ffsll((long long)zmask) - 1) {
                                    atomicAdd((unsigned long long*)&a.stats[ST_KEY0], (unsigned long long)__popcll(zmask));
                                    atomicOr((unsigned long long*)&a.stats[ST_KEY0_PRESENT], 1ull);
                                }
                            }
                            if (valid) my_valid++;
                        }
                        if constexpr (SINK == SINK_TABLE) {
                            bool done = true, claimed = false;
                            if (live) {
                                if constexpr (W == 1)
                                    done = insert_w1(key[0], a.table, a.cap, a.probe_limit, &claimed);
                                else
                                    done = insert_wide<W>(key, a.table, a.cap, a.probe_limit, &claimed);
                            }
                            u64 cm = __ballot(claimed);
                            if (cm && (int)lane_id() == __ffsll((long long)cm) - 1)
                                atomicAdd((unsigned long long*)&a.stats[ST_CLAIMED], (unsigned long long)__popcll(cm));
                            // spill: wave-aggregated reservation in the spill buffer
                            bool spill = !done;
                            if (__ballot(spill)) {
                                u64 idx = wave_reserve(&a.stats[ST_SPILL_FILL], spill);
                                if (spill) {
                                    if (idx < a.spill_cap) {
        #pragma unroll
                                        for (int j = 0; j < W; j++) a.spill[(u64)j * a.spill_cap + idx] = key[j];
                                    } else {
                                        atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_SPILL_OVERFLOW);
                                    }
                                }
                            }
                        }
                        // roll one base in
    #pragma unroll
                        for (int j = 0; j < W - 1; j++) raw[j] = (raw[j] << 2) | (raw[j + 1] >> 62);
                        raw[W - 1] = (raw[W - 1] << 2) | (tail >> 62);
                        tail <<= 2;
                    }
                }
            }
            __syncthreads();

            if constexpr (SINK == SINK_SCATTER) {
                // flush when the next tile might not fit, and at the segment end:
                // order the staged keys by digit through a permutation, then write
                // each digit's run with consecutive lanes
                const u32 n = s_misc[0];
                if (tile + 1 == t_end || n + (u32)pa.max_win > (u32)pa.scap) {
                    const u32 fmid = pa.out2 ? pa.fmid : 256u;
                    auto slot = [&](u64 k0) {
                        return ((u32)(k0 >> 56) >= fmid ? 256u : 0u) | ((u32)(k0 >> pa.shift) & 255u);
                    };
                    const u32 st = digit_scan256<512>(tid < 512 ? s_cnt[tid] : 0u, scan_tmp, tid);
                    if (tid < 512) {
                        s_fill[tid] = st;
                        s_gb[tid] = s_cur[tid] - st;
                    }
                    __syncthreads();
                    for (u32 i = tid; i < n; i += NT) {
                        u32 q = atomicAdd(&s_fill[slot(s_stage[i])], 1u);
                        s_perm[q] = (unsigned short)i;
                    }
                    __syncthreads();
                    for (u32 q = tid; q < n; q += NT) {
                        const u32 i = s_perm[q];
                        const u64 k0 = s_stage[i];
                        const u32 sl = slot(k0);
                        const u64 g = s_gb[sl] + q;
                        if (pa.skip & 1) continue;
                        u64* __restrict__ o = sl >= 256u ? pa.out2 : pa.out;
                        const u64 ost = sl >= 256u ? pa.out2_stride : pa.out_stride;
                        if (pa.aos) {
                            // one record per lane: a digit run is one contiguous
                            // stream, half the partial lines of two word arrays
                            if constexpr (W == 2) {
                                v2u64 v;
                                v.x = k0;
                                v.y = s_stage[(size_t)(pa.scap + 1) + i];
                                *(v2u64*)(o + 2 * g) = v;
                            } else {
                                o[g * W] = k0;
#pragma unroll
                                for (int j = 1; j < W; j++) o[g * W + j] = s_stage[(size_t)j * (pa.scap + 1) + i];
                            }
                        } else {
                            o[g] = k0;
#pragma unroll
                            for (int j = 1; j < W; j++) o[(u64)j * ost + g] = s_stage[(size_t)j * (pa.scap + 1) + i];
                        }
                        if (pa.digs) (sl >= 256u ? pa.digs2 : pa.digs)[g] = (unsigned char)(k0 >> 56);
                    }
                    __syncthreads();
                    if (tid < 512) {
                        s_cur[tid] += s_cnt[tid];
                        s_cnt[tid] = 0;
                    }
                    if (tid == 0) s_misc[0] = 0;
                    __syncthreads();
                }
            }
        }
        if constexpr (SINK == SINK_HIST) {
            __syncthreads();
            if (pa.gbits == 0) {
                for (int i = tid; i < 256; i += NT) pa.hist[(u64)i * pa.nseg + unit] = s_hist[i];
            } else {
                // grouped (key-range passes): the unit's bins contiguous, u32
                // (hist_group_sum_k transposes a pass's groups to digit-major)
                u32* h32 = (u32*)pa.hist + (u64)unit * (256u << pa.gbits);
                for (int i = tid; i < (256 << pa.gbits); i += NT) h32[i] = s_hist[i];
            }
            __syncthreads();
        }
    }
    if (SINK != SINK_HIST && !pa.no_stats) {
        wave_add(&a.stats[ST_VALID], my_valid);
        if (__ballot(my_hole) && lane_id() == 0) atomicOr((unsigned long long*)&a.stats[ST_KEY0_PRESENT], 1ull);
    }
}

static CountArgs make_args(const CountLaunch& l, const CountGeom& g) {
    CountArgs a;
    a.base = l.base;
    a.seq_off = l.seq_off;
    a.read0 = l.read0;
    a.n_reads = l.n_reads;
    a.L = l.L;
    a.k = l.k;
    a.R = g.R;
    a.NG = g.NG;
    a.raw_stride = g.raw_stride;
    a.table = l.table;
    a.cap = l.cap;
    a.spill = l.spill;
    a.spill_cap = l.spill_cap;
    a.stats = l.stats;
    a.probe_limit = l.probe_limit;
    a.rlen = l.rlen;
    return a;
}

#define KC_FRONT_SWITCH(SINKV, CODESV, NTV, GRID, LDS, S, A, PA)                                                     \
    switch (W) {                                                                                                     \
    case 1: hipLaunchKernelGGL((count_front<1, SINKV, CODESV, NTV>), dim3(GRID), dim3(NTV), LDS, S, A, PA); break;   \
    case 2: hipLaunchKernelGGL((count_front<2, SINKV, CODESV, NTV>), dim3(GRID), dim3(NTV), LDS, S, A, PA); break;   \
    case 3: hipLaunchKernelGGL((count_front<3, SINKV, CODESV, NTV>), dim3(GRID), dim3(NTV), LDS, S, A, PA); break;   \
    case 4: hipLaunchKernelGGL((count_front<4, SINKV, CODESV, NTV>), dim3(GRID), dim3(NTV), LDS, S, A, PA); break;   \
    default: return hipErrorInvalidValue;                                                                            \
    }

hipError_t launch_count_kmers(const CountLaunch& l, int grid_cap, hipStream_t s) {
    if (l.n_reads == 0) return hipSuccess;
    CountGeom g = count_geometry(l.L, l.k);
    CountArgs a = make_args(l, g);
    PartArgs pa;
    PartArgs zero_pa = {};
    pa = zero_pa;
    u64 tiles = (l.n_reads + g.R - 1) / g.R;
    int grid = (int)hmin(tiles, (u64)grid_cap);
    int W = (l.k + 31) / 32;
    KC_FRONT_SWITCH(SINK_TABLE, false, kBlock, grid, g.lds, s, a, pa)
    return hipGetLastError();
}

int groups_per_read(int L) { return (L + 15) / 16; }

// E: one thread per (read, 16-base group). Bytes past the read end encode as A
// with a clear mask bit, exactly as the LDS encoder of the text front end.
__global__ __launch_bounds__(kBlock) void encode_reads_k(const uint8_t* __restrict__ base,
                                                         const u64* __restrict__ seq_off, u64 read0, u64 n_reads,
                                                         int L, int G, u32* __restrict__ codes,
                                                         unsigned short* __restrict__ inval, u64* __restrict__ stats) {
    const u64 total = n_reads * (u64)G;
    bool hole = false;  // a not-ACGT base (stats[ST_VHOLE], when stats is given)
    for (u64 it = (u64)blockIdx.x * kBlock + threadIdx.x; it < total; it += (u64)gridDim.x * kBlock) {
        const u64 r = it / (u64)G;
        const int g = (int)(it - r * (u64)G);
        const u64 gr = read0 + r;
        const u64 off = (seq_off ? seq_off[gr] : gr * (u64)L) + 16 * (u64)g;
        const int nb = min(16, L - 16 * g);
        const uintptr_t addr = (uintptr_t)(base + off);
        // (global address space spelled out: the integer round trip would
        // otherwise leave FLAT loads)
        typedef __attribute__((address_space(1))) const u32 g32;
        const g32* dw = (const g32*)(addr & ~(uintptr_t)3);
        const int sh = (int)(addr & 3);
        // only dwords holding a byte of this group are read (no load past the text)
        u32 d[5];
        if (sh + nb > 12) {
            // the first four dwords in one (4-byte aligned) 16-byte load
            typedef v4u v4u_a4 __attribute__((aligned(4)));
            const v4u q = __builtin_nontemporal_load((const __attribute__((address_space(1))) v4u_a4*)dw);
            d[0] = q.x;
            d[1] = q.y;
            d[2] = q.z;
            d[3] = q.w;
            d[4] = (16 < sh + nb) ? __builtin_nontemporal_load(dw + 4) : 0u;
        } else {
#pragma unroll
            for (int i = 0; i < 5; i++) d[i] = (4 * i < sh + nb) ? __builtin_nontemporal_load(dw + i) : 0u;
        }
        const u32 x0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
        const u32 x1 = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
        const u32 x2 = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
        const u32 x3 = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
        u32 b0, b1, b2, b3;
        const u32 c0 = bytes_to_codes(x0, nb, &b0);
        const u32 c1 = bytes_to_codes(x1, nb - 4, &b1);
        const u32 c2 = bytes_to_codes(x2, nb - 8, &b2);
        const u32 c3 = bytes_to_codes(x3, nb - 12, &b3);
        codes[it] = (c0 << 24) | (c1 << 16) | (c2 << 8) | c3;
        const u32 bad = (b0 << 12) | (b1 << 8) | (b2 << 4) | b3;
        inval[it] = (unsigned short)bad;
        hole = hole || bad != 0u;
    }
    if (stats && __ballot(hole) && lane_id() == 0) atomicOr((unsigned long long*)&stats[ST_VHOLE], 1ull);
}

hipError_t launch_encode_reads(const CountLaunch& l, uint32_t* codes, uint16_t* inval, hipStream_t s, uint64_t* stats) {
    if (l.n_reads == 0) return hipSuccess;
    const int G = groups_per_read(l.L);
    const u64 total = l.n_reads * (u64)G;
    const int grid = (int)hmin((total + kBlock - 1) / kBlock, 65536);
    hipLaunchKernelGGL(encode_reads_k, dim3(grid), dim3(kBlock), 0, s, l.base, l.seq_off, l.read0, l.n_reads, l.L, G,
                       codes, (unsigned short*)inval, (u64*)stats);
    return hipGetLastError();
}

// E for variable-length reads (KC_FLAG_VARLEN): one thread per (read, 16-base
// group) of an L-base slot; the read's own bytes as in encode_reads_k, the
// slot past its end marked not-ACGT with code 0, so the read counts exactly
// the windows of a reference read of its own length (GPUHandler.cu:129-233 at
// L = its length: a window needs k valid bases, key bases past the end are 0)
__global__ __launch_bounds__(kBlock) void encode_reads_var_k(const uint8_t* __restrict__ base,
                                                             const u64* __restrict__ seq_off,
                                                             const u64* __restrict__ seq_end, u64 n_reads, int L,
                                                             int G, int k, u32* __restrict__ codes,
                                                             unsigned short* __restrict__ inval,
                                                             unsigned short* __restrict__ rlen, u64* stats) {
    const u64 total = n_reads * (u64)G;
    bool too_long = false, hole = false;
    u64 win = 0;
    for (u64 it = (u64)blockIdx.x * kBlock + threadIdx.x; it < total; it += (u64)gridDim.x * kBlock) {
        const u64 r = it / (u64)G;
        const int g = (int)(it - r * (u64)G);
        const u64 s0 = seq_off[r];
        const u64 len = seq_end[r] - s0;
        if (len > (u64)L) {
            too_long = true;
            codes[it] = 0u;
            inval[it] = 0xffffu;
            if (rlen && g == 0) rlen[r] = 0;
            continue;
        }
        if (rlen && g == 0) rlen[r] = (unsigned short)len;
        if (g == 0 && len >= (u64)k) win += len - (u64)k + 1;
        const int nb = min(16, L - 16 * g);                            // bases of the slot in this group
        const int nr = max(0, min(nb, (int)len - 16 * g));             // of them, bases of the read
        u32 d[5] = {0u, 0u, 0u, 0u, 0u};
        int sh = 0;
        if (nr > 0) {
            const uintptr_t addr = (uintptr_t)(base + s0 + 16 * (u64)g);
            typedef __attribute__((address_space(1))) const u32 g32;
            const g32* dw = (const g32*)(addr & ~(uintptr_t)3);
            sh = (int)(addr & 3);
#pragma unroll
            for (int i = 0; i < 5; i++) d[i] = (4 * i < sh + nr) ? __builtin_nontemporal_load(dw + i) : 0u;
        }
        const u32 x0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
        const u32 x1 = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
        const u32 x2 = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
        const u32 x3 = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
        u32 b0, b1, b2, b3;
        const u32 c0 = bytes_to_codes(x0, nr, &b0);
        const u32 c1 = bytes_to_codes(x1, nr - 4, &b1);
        const u32 c2 = bytes_to_codes(x2, nr - 8, &b2);
        const u32 c3 = bytes_to_codes(x3, nr - 12, &b3);
        const u32 bad = (b0 << 12) | (b1 << 8) | (b2 << 4) | b3;
        if (bad != 0u && len >= (u64)k) hole = true;
        // slot positions [nr, nb) lie past the read: bits 15 - i
        const u32 pad = ((1u << (16 - nr)) - 1u) & ~((1u << (16 - nb)) - 1u);
        codes[it] = (c0 << 24) | (c1 << 16) | (c2 << 8) | c3;
        inval[it] = (unsigned short)(bad | pad);
    }
    if (__ballot(too_long) && lane_id() == 0) atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)ERR_FQ_SEQ_LEN);
    if (__ballot(hole) && lane_id() == 0) atomicOr((unsigned long long*)&stats[ST_VHOLE], 1ull);
    for (int o = 32; o >= 1; o >>= 1) win += __shfl_xor(win, o);
    if (lane_id() == 0 && win) atomicAdd((unsigned long long*)&stats[ST_VWIN], (unsigned long long)win);
}

hipError_t launch_encode_reads_var(const uint8_t* base, const uint64_t* seq_off, const uint64_t* seq_end,
                                   uint64_t n_reads, int L, int k, uint32_t* codes, uint16_t* inval, uint16_t* rlen,
                                   uint64_t* stats, hipStream_t s) {
    if (n_reads == 0) return hipSuccess;
    if (L < 1 || k < 1) return hipErrorInvalidValue;
    const int G = groups_per_read(L);
    const u64 total = n_reads * (u64)G;
    const int grid = (int)hmin((total + kBlock - 1) / kBlock, 65536);
    hipLaunchKernelGGL(encode_reads_var_k, dim3(grid), dim3(kBlock), 0, s, base, (const u64*)seq_off,
                       (const u64*)seq_end, n_reads, L, G, k, codes, (unsigned short*)inval, (unsigned short*)rlen,
                       (u64*)stats);
    return hipGetLastError();
}

// P2 workgroup: kP2Block threads, one per CU, most of the CU's LDS for staging
constexpr int kP2Block = 1024;
constexpr size_t kPartLds = 160 * 1024 - 512;  // the P2 workgroup's LDS (front + sink, with alignment) stays under 160 KiB

PartGeom part_geometry(int L, int k, uint64_t n_reads) {
    PartGeom p;
    CountGeom g = count_geometry(L, k);
    g.raw_stride = 0;  // CODES front end: no raw text in LDS
    // aim for two rounds of 8-window runs per P2 thread; the P1 workgroup
    // (256 threads) walks the same tiles in more rounds
    const int nw0 = L - k + 1;
    g.R = (2 * kP2Block * 8 + nw0 - 1) / (nw0 > 0 ? nw0 : 1);
    if (g.R > 256) g.R = 256;
    if (g.R < 1) g.R = 1;
    while (g.R > 1 && g.R * g.NG > kPrefetch * kBlock) g.R--;
    // P1 and P2 share this tile geometry. P2 stages keys over several tiles
    // (scap >= 2 tiles where possible) before writing them in digit order, so
    // each digit run written is long enough to fill whole cache lines.
    const int W = (k + 31) / 32;
    const int nw = L - k + 1;
    auto front = [&](int r) {
        size_t f = (size_t)r * g.raw_stride + (size_t)r * g.NG * 8 + (size_t)r * 8 + 16;
        return ((f + 15) & ~(size_t)15) + 16;
    };
    const size_t per_key = (size_t)W * 8 + 2;  // staged key words + u16 permutation entry
    while (g.R > 1 && front(g.R) + sink_lds_host(W, SINK_SCATTER, 2 * g.R * nw) > kPartLds) g.R--;
    g.R = balance_reads(g.R, nw, kP2Block);
    // staging room: what the front end and the sink's fixed arrays (slot
    // cursors and counters, sink_lds_host at scap = 0) leave
    const size_t fixed = sink_lds_host(W, SINK_SCATTER, 0) + 64;
    size_t room = kPartLds > front(g.R) + fixed ? kPartLds - front(g.R) - fixed : 0;
    int scap = (int)(room / per_key);
    if (scap > 65535) scap = 65535;  // u16 permutation indices
    if (scap < g.R * nw) scap = g.R * nw;
    g.lds = (((size_t)g.R * g.raw_stride + (size_t)g.R * g.NG * 8 + (size_t)g.R * 8 + 16) + 15) & ~(size_t)15;
    p.geom = g;
    u64 tiles = (n_reads + g.R - 1) / g.R;
    u64 seg_tiles = (tiles + 16383) / 16384;
    if (seg_tiles < 4) seg_tiles = 4;
    p.seg_tiles = (int)seg_tiles;
    p.nseg = (tiles + seg_tiles - 1) / seg_tiles;
    p.max_win = g.R * nw;
    p.scap = scap;
    p.lds_scatter = ((g.lds + 15) & ~(size_t)15) + 16 + sink_lds_host(W, SINK_SCATTER, scap);  // as launched
    return p;
}

hipError_t launch_part_hist(const CountLaunch& l, const PartGeom& pg, uint64_t* hist, int shift, hipStream_t s,
                            int gbits) {
    if (gbits < 0 || gbits > 4) return hipErrorInvalidValue;
    if (l.n_reads == 0) return hipSuccess;
    const CountGeom& g = pg.geom;
    CountArgs a = make_args(l, g);
    int W = (l.k + 31) / 32;
    PartArgs pa;
    PartArgs zero_pa = {};
    pa = zero_pa;
    pa.hist = hist;
    pa.codes = l.codes;
    pa.inval = (const unsigned short*)l.inval;
    pa.G = groups_per_read(l.L);
    if (!l.codes || !l.inval) return hipErrorInvalidValue;
    pa.nseg = pg.nseg;
    pa.seg_tiles = pg.seg_tiles;
    pa.flo = l.flo;
    pa.fhi = l.fhi;
    pa.no_stats = l.no_stats ? 1 : 0;
    pa.gbits = gbits;
    pa.shift = shift;
    pa.max_win = pg.max_win;
    pa.scap = pg.scap;
    size_t lds = ((g.lds + 15) & ~(size_t)15) + 16 + ((size_t)256 << gbits) * 4;
    int grid = (int)hmin(pg.nseg, 4096);
    KC_FRONT_SWITCH(SINK_HIST, true, kBlock, grid, lds, s, a, pa)
    return hipGetLastError();
}

hipError_t launch_part_scatter(const CountLaunch& l, const PartGeom& pg, const uint64_t* base, uint64_t* out,
                               uint64_t out_stride, int shift, uint8_t* digs, hipStream_t s, const uint64_t* base2,
                               uint64_t* out2, uint64_t out2_stride, uint8_t* digs2, uint32_t fmid, bool aos) {
    if (l.n_reads == 0) return hipSuccess;
    const CountGeom& g = pg.geom;
    CountArgs a = make_args(l, g);
    int W = (l.k + 31) / 32;
    PartArgs pa;
    PartArgs zero_pa = {};
    pa = zero_pa;
    pa.base = base;
    pa.out = out;
    pa.digs = (unsigned char*)digs;
    pa.aos = aos ? 1 : 0;
    pa.out_stride = out_stride;
    pa.codes = l.codes;
    pa.inval = (const unsigned short*)l.inval;
    pa.G = groups_per_read(l.L);
    if (!l.codes || !l.inval) return hipErrorInvalidValue;
    pa.nseg = pg.nseg;
    pa.seg_tiles = pg.seg_tiles;
    pa.flo = l.flo;
    pa.fhi = l.fhi;
    pa.no_stats = l.no_stats ? 1 : 0;
    if (out2 && (!base2 || (!digs2 && digs) || fmid <= l.flo || fmid >= l.fhi)) return hipErrorInvalidValue;
    pa.out2 = out2;
    pa.out2_stride = out2_stride;
    pa.base2 = base2;
    pa.digs2 = (unsigned char*)digs2;
    pa.fmid = fmid;
    pa.shift = shift;
    pa.max_win = pg.max_win;
    pa.scap = pg.scap;
    pa.skip = experiment_knob("KC_P2_SKIP");
    size_t lds = ((g.lds + 15) & ~(size_t)15) + 16 + sink_lds_host(W, SINK_SCATTER, pg.scap);
    int grid = (int)hmin(pg.nseg, 4096);
    KC_FRONT_SWITCH(SINK_SCATTER, true, kP2Block, grid, lds, s, a, pa)
    return hipGetLastError();
}

// Key-range passes: a P1 histogram of 16 groups (word0 >> 60) x 256 digits
// per segment (launch_part_hist, gbits = 4) gives every pass its digit x
// segment histogram without walking the reads again (groups [g0, g1)
// summed), and the planner its group totals.
__global__ __launch_bounds__(kBlock) void hist_group_sum_k(const u32* __restrict__ h, u64 nseg, u32 g0, u32 g1,
                                                           u64* __restrict__ out) {
    // h: per segment 4096 u32 bins (group g, digit d at g * 256 + d); out:
    // the pass's digit-major histogram out[d * nseg + seg]. 32 segments per
    // step through an LDS tile: loads contiguous per segment, stores 32
    // consecutive segments of one digit
    __shared__ u32 tile[256][33];
    const int tid = threadIdx.x;
    for (u64 s0 = (u64)blockIdx.x * 32; s0 < nseg; s0 += (u64)gridDim.x * 32) {
        const u32 ns = (u32)min((u64)32, nseg - s0);
        for (u32 j = 0; j < ns; j++) {
            const u32* hs = h + (s0 + j) * 4096u;
            u32 v = 0;
            for (u32 g = g0; g < g1; g++) v += hs[g * 256u + (u32)tid];
            tile[tid][j] = v;
        }
        __syncthreads();
        for (u32 x = (u32)tid; x < 256u * 32u; x += kBlock) {
            const u32 d = x >> 5, j = x & 31u;
            if (j < ns) out[(u64)d * nseg + s0 + j] = tile[d][j];
        }
        __syncthreads();
    }
}

// group totals (tot zeroed by the caller): thread t holds bin t of every
// group for the block's segments, summed per group across the block
__global__ __launch_bounds__(kBlock) void hist_group_totals_k(const u32* __restrict__ h, u64 nseg,
                                                              u64* __restrict__ tot) {
    __shared__ u64 part[16][kBlock / 64];
    u64 v[16];
#pragma unroll
    for (int g = 0; g < 16; g++) v[g] = 0;
    for (u64 sg = blockIdx.x; sg < nseg; sg += gridDim.x) {
        const u32* hs = h + sg * 4096u + threadIdx.x;
#pragma unroll
        for (int g = 0; g < 16; g++) v[g] += hs[g * 256];
    }
#pragma unroll
    for (int g = 0; g < 16; g++) {
        u64 x = v[g];
        for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
        if (lane_id() == 0) part[g][threadIdx.x >> 6] = x;
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        u64 t = 0;
        for (int w = 0; w < kBlock / 64; w++) t += part[threadIdx.x][w];
        if (t) atomicAdd((unsigned long long*)&tot[threadIdx.x], (unsigned long long)t);
    }
}

hipError_t launch_hist_group_sum(const uint64_t* h, uint64_t nseg, uint32_t g0, uint32_t g1, uint64_t* out,
                                 hipStream_t s) {
    if (g1 > 16 || g0 >= g1) return hipErrorInvalidValue;
    const int grid = (int)hmin((nseg + 31) / 32, 4096);
    hipLaunchKernelGGL(hist_group_sum_k, dim3(grid), dim3(kBlock), 0, s, (const u32*)h, (u64)nseg, g0, g1, (u64*)out);
    return hipGetLastError();
}

hipError_t launch_hist_group_totals(const uint64_t* h, uint64_t nseg, uint32_t groups, uint64_t* tot, hipStream_t s) {
    if (groups != 16) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(tot, 0, 16 * 8, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(hist_group_totals_k, dim3((u32)hmin(nseg, 1024)), dim3(kBlock), 0, s, (const u32*)h, (u64)nseg,
                       (u64*)tot);
    return hipGetLastError();
}

#undef KC_FRONT_SWITCH

// ---------------------------------------------------------------------------
// K3: compact — occupied slots -> dense SoA records (order is arbitrary; the
// radix sort fixes it).
// ---------------------------------------------------------------------------

template <typename T>
static hipError_t scan_impl(const T* in, T* out, u64 n, T* tmp, hipStream_t s);

__global__ void sum_last(const u64* base, const u64* counts, u64 n, u64* out) { *out = base[n - 1] + counts[n - 1]; }

hipError_t launch_sum_last(const uint64_t* base, const uint64_t* counts, uint64_t n, uint64_t* out, hipStream_t s) {
    if (n == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sum_last, dim3(1), dim3(1), 0, s, base, counts, (u64)n, out);
    return hipGetLastError();
}

constexpr int kCompactGrid = 4096;

__device__ __forceinline__ void compact_range(u64 cap, int grid, int b, u64* lo, u64* hi) {
    u64 per = ((cap + grid - 1) / grid + kBlock - 1) / kBlock * kBlock;
    *lo = min(cap, (u64)b * per);
    *hi = min(cap, *lo + per);
}

template <int W>
__device__ __forceinline__ bool slot_occupied(const u64* slot) {
    if constexpr (W == 1)
        return slot[0] != 0ull;
    else
        return (u32)(slot[W] >> 32) == 2u;
}

// pass 1: occupied slots per block range
template <int W>
__global__ __launch_bounds__(kBlock) void compact_count(const u64* __restrict__ table, u64 cap,
                                                        u64* __restrict__ block_counts) {
    constexpr int SW = (W == 1) ? 2 : ((W <= 3) ? 4 : 8);
    __shared__ u32 part[4];
    u64 lo, hi;
    compact_range(cap, gridDim.x, blockIdx.x, &lo, &hi);
    u32 cnt = 0;
    for (u64 s = lo + threadIdx.x; s < hi; s += kBlock) cnt += slot_occupied<W>(table + SW * s) ? 1u : 0u;
    for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (lane_id() == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) block_counts[blockIdx.x] = (u64)part[0] + part[1] + part[2] + part[3];
}

// pass 2: write occupied slots in slot order at the scanned block offsets
template <int W>
__global__ __launch_bounds__(kBlock) void compact_emit(const u64* __restrict__ table, u64 cap,
                                                       const u64* __restrict__ block_base, u64* __restrict__ keys,
                                                       u32* __restrict__ cnts, u64 out_cap) {
    constexpr int SW = (W == 1) ? 2 : ((W <= 3) ? 4 : 8);
    __shared__ u32 scan_tmp[4];
    u64 lo, hi;
    compact_range(cap, gridDim.x, blockIdx.x, &lo, &hi);
    u64 run = block_base[blockIdx.x];
    for (u64 b = lo; b < hi; b += kBlock) {
        u64 s = b + threadIdx.x;
        bool occ = false;
        u64 kw[W];
        u32 c = 0;
        if (s < hi) {
            const u64* slot = table + SW * s;
#pragma unroll
            for (int j = 0; j < W; j++) kw[j] = slot[j];
            c = (u32)slot[W];
            occ = slot_occupied<W>(slot);
        }
        u32 total;
        u32 before = block_excl_scan(occ ? 1u : 0u, scan_tmp, &total);
        if (occ) {
            u64 pos = run + before;
            if (pos < out_cap) {
#pragma unroll
                for (int j = 0; j < W; j++) keys[(u64)j * out_cap + pos] = kw[j];
                cnts[pos] = c;
            }
        }
        run += total;
    }
}

template <int W>
__global__ void append_key0(u64* keys, u32* cnts, u64 out_cap, u64* cursor, const u64* stats) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (stats[ST_KEY0_PRESENT] == 0) return;
    u64 pos = *cursor;
    if (pos >= out_cap) return;
    for (int j = 0; j < W; j++) keys[(u64)j * out_cap + pos] = 0ull;
    cnts[pos] = (u32)stats[ST_KEY0];
    *cursor = pos + 1;
}

hipError_t launch_compact(int W, const uint64_t* table, uint64_t cap, uint64_t* keys, uint32_t* cnts,
                          uint64_t out_cap, uint64_t* cursor, uint64_t* tmp, hipStream_t s) {
    // tmp: kCompactGrid block counts + kCompactGrid offsets + 1 scan partial
    int grid = kCompactGrid;
    u64* counts = tmp;
    u64* base = tmp + kCompactGrid;
    u64* stmp = tmp + 2 * kCompactGrid;
#define KC_CC(WW) hipLaunchKernelGGL(compact_count<WW>, dim3(grid), dim3(kBlock), 0, s, table, cap, counts)
#define KC_CE(WW) hipLaunchKernelGGL(compact_emit<WW>, dim3(grid), dim3(kBlock), 0, s, table, cap, (const u64*)base, keys, cnts, out_cap)
    switch (W) {
    case 1: KC_CC(1); break;
    case 2: KC_CC(2); break;
    case 3: KC_CC(3); break;
    case 4: KC_CC(4); break;
    default: return hipErrorInvalidValue;
    }
    hipError_t e = scan_impl<u64>(counts, base, (u64)grid, stmp, s);
    if (e != hipSuccess) return e;
    switch (W) {
    case 1: KC_CE(1); break;
    case 2: KC_CE(2); break;
    case 3: KC_CE(3); break;
    case 4: KC_CE(4); break;
    }
#undef KC_CC
#undef KC_CE
    // cursor = total occupied = base[grid-1] + counts[grid-1]
    hipLaunchKernelGGL(sum_last, dim3(1), dim3(1), 0, s, base, counts, (u64)grid, cursor);
    return hipGetLastError();
}

uint64_t compact_tmp_elems() { return 2 * kCompactGrid + scan_tmp_elems(kCompactGrid) + 8; }

hipError_t launch_append_key0(int W, uint64_t* keys, uint32_t* cnts, uint64_t out_cap, uint64_t* cursor,
                              const uint64_t* stats, hipStream_t s) {
    switch (W) {
    case 1: hipLaunchKernelGGL(append_key0<1>, dim3(1), dim3(64), 0, s, keys, cnts, out_cap, cursor, stats); break;
    case 2: hipLaunchKernelGGL(append_key0<2>, dim3(1), dim3(64), 0, s, keys, cnts, out_cap, cursor, stats); break;
    case 3: hipLaunchKernelGGL(append_key0<3>, dim3(1), dim3(64), 0, s, keys, cnts, out_cap, cursor, stats); break;
    case 4: hipLaunchKernelGGL(append_key0<4>, dim3(1), dim3(64), 0, s, keys, cnts, out_cap, cursor, stats); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K4: LSD radix sort (8-bit digits) of SoA records, stable. Per pass:
//   upsweep   : per-block digit histogram -> hist[d * grid + b]
//   scan      : single-block exclusive scan of hist (digit-major)
//   downsweep : per 2048-record tile, stable in-tile ranking (wave match via 8
//               ballots + cross-wave prefix in LDS), records permuted through
//               LDS into digit order, then written to their global positions.
// ---------------------------------------------------------------------------

constexpr int kSortItems = 8;
constexpr int kSortTile = kBlock * kSortItems;  // 2048 (grid sizing granule)

template <int W>
struct SortCfg {
    static constexpr int ITEMS = (W == 1) ? 16 : ((W == 2) ? 8 : 4);  // rounds per wave
    static constexpr int TILE = 4 * 64 * ITEMS;
};

uint64_t sort_hist_elems(int grid) { return (u64)256 * grid + scan_tmp_elems((u64)256 * grid) + 16; }  // u64

int sort_grid(uint64_t n) {
    u64 tiles = (n + kSortTile - 1) / kSortTile;
    u64 g = tiles < 2048 ? tiles : 2048;
    return (int)(g ? g : 1);
}

__device__ __forceinline__ void block_range(u64 n, int grid, int b, u64* lo, u64* hi) {
    u64 tiles = (n + kSortTile - 1) / kSortTile;
    u64 per = (tiles + grid - 1) / grid;
    *lo = min(n, (u64)b * per * kSortTile);
    *hi = min(n, (u64)(b + 1) * per * kSortTile);
}

template <int W, bool HASHED>
__device__ __forceinline__ u32 sort_digit(const u64 (&k)[W], int word, int shift) {
    u64 dw;
    if constexpr (HASHED) {
        dw = hash_key<W>(k);
    } else {
        dw = k[0];
#pragma unroll
        for (int j = 1; j < W; j++)
            if (j == word) dw = k[j];
    }
    return (u32)(dw >> shift) & 255u;
}

template <int W, bool HASHED>
__global__ __launch_bounds__(kBlock) void sort_upsweep(const u64* __restrict__ keys, u64 stride, u64 n, int word,
                                                       int shift, u64* __restrict__ hist) {
    __shared__ u32 h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    u64 lo, hi;
    {
        constexpr int TILE = SortCfg<W>::TILE;
        u64 tiles = (n + TILE - 1) / TILE;
        u64 per = (tiles + gridDim.x - 1) / gridDim.x;
        lo = min(n, (u64)blockIdx.x * per * TILE);
        hi = min(n, (u64)(blockIdx.x + 1) * per * TILE);
    }
    for (u64 i = lo + threadIdx.x; i < hi; i += kBlock) {
        u64 k[W];
        if constexpr (HASHED) {
#pragma unroll
            for (int j = 0; j < W; j++) k[j] = keys[(u64)j * stride + i];
        } else {
#pragma unroll
            for (int j = 0; j < W; j++) k[j] = (j == word) ? keys[(u64)j * stride + i] : 0ull;
        }
        atomicAdd(&h[sort_digit<W, HASHED>(k, word, shift)], 1u);
    }
    __syncthreads();
    hist[(u64)threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

// Downsweep with wave-private stable ranking. A tile of kSortTile records is
// split into 4 contiguous quarters, one per wave; a wave walks its quarter in
// rounds of 64 consecutive records, finds the lanes sharing its digit with 8
// ballots, and ranks them against its own running per-digit counters in LDS
// (only that wave touches its row, so no barrier is needed between rounds).
// One block-wide prefix over (digit, wave) then gives every record its stable
// position in the tile; records are permuted through LDS and written out in
// digit runs.
template <int W, bool HAS_VALS, bool HASHED>
__global__ __launch_bounds__(kBlock) void sort_downsweep(const u64* __restrict__ kin, u64* __restrict__ kout,
                                                         const u32* __restrict__ vin, u32* __restrict__ vout,
                                                         u64 stride, u64 n, int word, int shift,
                                                         const u64* __restrict__ hist) {
    constexpr int ITEMS = SortCfg<W>::ITEMS;
    constexpr int TILE = SortCfg<W>::TILE;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64* skeys = (u64*)smem;                          // W x TILE
    u32* svals = (u32*)(skeys + W * TILE);            // TILE (only with values)
    u32* wcnt = svals + (HAS_VALS ? TILE : 0);        // 4 x 256 running counts per wave
    u32* woff = wcnt + 4 * 256;                       // 4 x 256 offsets of a wave inside a digit
    u32* dtot = woff + 4 * 256;                       // 256 digit totals of the tile
    u32* dstart = dtot + 256;                         // 256 tile-local digit starts
    u32* scan_tmp = dstart + 256;                     // 4 (+4 pad)
    u64* global_off = (u64*)(scan_tmp + 8);           // 256 running global offsets

    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    global_off[tid] = hist[(u64)tid * gridDim.x + blockIdx.x];
    for (int i = tid; i < 4 * 256; i += kBlock) wcnt[i] = 0;
    __syncthreads();

    u64 lo, hi;
    {
        u64 tiles = (n + TILE - 1) / TILE;
        u64 per = (tiles + gridDim.x - 1) / gridDim.x;
        lo = min(n, (u64)blockIdx.x * per * TILE);
        hi = min(n, (u64)(blockIdx.x + 1) * per * TILE);
    }
    const u64 lanemask = lanemask_lt();
    for (u64 t0 = lo; t0 < hi; t0 += TILE) {
        u64 kreg[ITEMS][W];
        u32 vreg[ITEMS];
        u32 dreg[ITEMS];
        u32 rank[ITEMS];
        const u64 q0 = t0 + (u64)wave * (64 * ITEMS) + lane;
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const u64 i = min(q0 + (u64)it * 64, hi - 1);  // unconditional loads (clamped)
#pragma unroll
            for (int j = 0; j < W; j++) kreg[it][j] = kin[(u64)j * stride + i];
            if constexpr (HAS_VALS) vreg[it] = vin[i];
        }
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            u64 i = q0 + (u64)it * 64;
            bool ok = i < hi;
            u32 d = sort_digit<W, HASHED>(kreg[it], word, shift);
            dreg[it] = d;
            u64 peers = __ballot(ok);
#pragma unroll
            for (int b = 0; b < 8; b++) {
                u64 bb = __ballot((d >> b) & 1u);
                peers &= ((d >> b) & 1u) ? bb : ~bb;
            }
            u32 before = (u32)__popcll(peers & lanemask);
            u32 base = ok ? wcnt[wave * 256 + d] : 0u;
            // all lanes have read the counter; the group's lowest lane bumps it
            if (ok && before == 0) wcnt[wave * 256 + d] = base + (u32)__popcll(peers);
            rank[it] = ok ? base + before : 0xffffffffu;
        }
        __syncthreads();
        {
            u32 run = 0;
#pragma unroll
            for (int w = 0; w < 4; w++) {
                u32 c = wcnt[w * 256 + tid];
                woff[w * 256 + tid] = run;
                wcnt[w * 256 + tid] = 0;
                run += c;
            }
            dtot[tid] = run;
            u32 total;
            dstart[tid] = block_excl_scan(run, scan_tmp, &total);
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            if (rank[it] == 0xffffffffu) continue;
            u32 d = dreg[it];
            u32 pos = dstart[d] + woff[wave * 256 + d] + rank[it];
#pragma unroll
            for (int j = 0; j < W; j++) skeys[j * TILE + pos] = kreg[it][j];
            if constexpr (HAS_VALS) svals[pos] = vreg[it];
        }
        __syncthreads();
        const u32 m = (u32)min((u64)TILE, hi - t0);
        for (u32 pos = tid; pos < m; pos += kBlock) {
            u64 k0[W];
#pragma unroll
            for (int j = 0; j < W; j++) k0[j] = skeys[j * TILE + pos];
            u32 d = sort_digit<W, HASHED>(k0, word, shift);
            u64 g = global_off[d] + (pos - dstart[d]);
#pragma unroll
            for (int j = 0; j < W; j++) kout[(u64)j * stride + g] = k0[j];
            if constexpr (HAS_VALS) vout[g] = svals[pos];
        }
        __syncthreads();
        global_off[tid] += dtot[tid];
    }
}

hipError_t launch_sort_pass(int W, const uint64_t* keys_in, uint64_t* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, uint64_t stride, uint64_t n, int word, int shift, uint64_t* hist,
                            int grid, bool hashed, hipStream_t s) {
    if (n == 0) return hipSuccess;
#define KC_UP(WW, HH) hipLaunchKernelGGL((sort_upsweep<WW, HH>), dim3(grid), dim3(kBlock), 0, s, keys_in, stride, n, word, shift, hist)
    switch (W * 2 + (hashed ? 1 : 0)) {
    case 2: KC_UP(1, false); break;
    case 3: KC_UP(1, true); break;
    case 4: KC_UP(2, false); break;
    case 5: KC_UP(2, true); break;
    case 6: KC_UP(3, false); break;
    case 7: KC_UP(3, true); break;
    case 8: KC_UP(4, false); break;
    case 9: KC_UP(4, true); break;
    default: return hipErrorInvalidValue;
    }
#undef KC_UP
    {
        hipError_t e = scan_impl<u64>(hist, hist, (u64)256 * grid, hist + (u64)256 * grid, s);
        if (e != hipSuccess) return e;
    }
    const int tile = 4 * 64 * ((W == 1) ? 16 : ((W == 2) ? 8 : 4));
    size_t lds = (size_t)W * tile * 8 + (vals_in ? (size_t)tile * 4 : 0) + (8 * 256 + 2 * 256 + 8) * 4 + 256 * 8;
    lds = (lds + 15) & ~(size_t)15;
    bool hv = vals_in != nullptr;
#define KC_DOWN(WW, HV, HH)                                                                                      \
    hipLaunchKernelGGL((sort_downsweep<WW, HV, HH>), dim3(grid), dim3(kBlock), lds, s, keys_in, keys_out, vals_in, \
                       vals_out, stride, n, word, shift, (const u64*)hist)
#define KC_DOWN_W(WW)                           \
    case WW:                                    \
        if (hv && hashed) KC_DOWN(WW, true, true);       \
        else if (hv) KC_DOWN(WW, true, false);           \
        else if (hashed) KC_DOWN(WW, false, true);       \
        else KC_DOWN(WW, false, false);                  \
        break;
    switch (W) {
        KC_DOWN_W(1)
        KC_DOWN_W(2)
        KC_DOWN_W(3)
        KC_DOWN_W(4)
    default: return hipErrorInvalidValue;
    }
#undef KC_DOWN_W
#undef KC_DOWN
    return hipGetLastError();
}

template <int W>
__global__ __launch_bounds__(kBlock) void key_bits(const u64* __restrict__ keys, u64 stride, u64 n, u64* bits) {
    u64 o[W], a[W];
#pragma unroll
    for (int j = 0; j < W; j++) {
        o[j] = 0;
        a[j] = ~0ull;
    }
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
#pragma unroll
        for (int j = 0; j < W; j++) {
            u64 v = keys[(u64)j * stride + i];
            o[j] |= v;
            a[j] &= v;
        }
    }
#pragma unroll
    for (int j = 0; j < W; j++) {
        for (int s = 32; s >= 1; s >>= 1) {
            o[j] |= __shfl_xor(o[j], s);
            a[j] &= __shfl_xor(a[j], s);
        }
        if (lane_id() == 0) {
            atomicOr((unsigned long long*)&bits[j], o[j]);
            atomicAnd((unsigned long long*)&bits[W + j], a[j]);
        }
    }
}

hipError_t launch_key_bits(int W, const uint64_t* keys, uint64_t stride, uint64_t n, uint64_t* bits, hipStream_t s) {
    int grid = (int)hmin((n + kBlock - 1) / kBlock, 2048);
    if (grid < 1) grid = 1;
    switch (W) {
    case 1: hipLaunchKernelGGL(key_bits<1>, dim3(grid), dim3(kBlock), 0, s, keys, stride, n, bits); break;
    case 2: hipLaunchKernelGGL(key_bits<2>, dim3(grid), dim3(kBlock), 0, s, keys, stride, n, bits); break;
    case 3: hipLaunchKernelGGL(key_bits<3>, dim3(grid), dim3(kBlock), 0, s, keys, stride, n, bits); break;
    case 4: hipLaunchKernelGGL(key_bits<4>, dim3(grid), dim3(kBlock), 0, s, keys, stride, n, bits); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// device-wide exclusive scan (reduce -> single-block scan -> downsweep)
// ---------------------------------------------------------------------------

constexpr int kScanItems = 16;
constexpr int kScanTile = kBlock * kScanItems;  // 4096

uint64_t scan_tmp_elems(uint64_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

template <typename T>
__global__ __launch_bounds__(kBlock) void scan_reduce(const T* __restrict__ in, u64 n, T* __restrict__ sums) {
    __shared__ T part[kBlock / kWave];
    u64 base = (u64)blockIdx.x * kScanTile;
    T s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        u64 idx = base + (u64)i * kBlock + threadIdx.x;
        if (idx < n) s += in[idx];
    }
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane_id() == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) sums[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

template <typename T>
__global__ __launch_bounds__(1024) void scan_single(T* data, u64 m) {
    __shared__ T part[1024];
    const int t = threadIdx.x;
    u64 per = (m + 1023) / 1024;
    u64 lo = min(m, (u64)t * per), hi = min(m, lo + per);
    T sum = 0;
    for (u64 i = lo; i < hi; i++) sum += data[i];
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        T v = (t >= o) ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    T run = part[t] - sum;
    for (u64 i = lo; i < hi; i++) {
        T v = data[i];
        data[i] = run;
        run += v;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void scan_down(const T* __restrict__ in, T* __restrict__ out, u64 n,
                                                    const T* __restrict__ sums) {
    __shared__ T wsum[kBlock / kWave];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    // blocked: thread t owns items base + t*kScanItems .. +kScanItems
    u64 base = (u64)blockIdx.x * kScanTile + (u64)tid * kScanItems;
    T v[kScanItems];
    T s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        u64 idx = base + i;
        v[i] = idx < n ? in[idx] : (T)0;
        s += v[i];
    }
    T x = s;
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    T before = sums[blockIdx.x];
    for (int w = 0; w < wave; w++) before += wsum[w];
    T run = before + x - s;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        u64 idx = base + i;
        if (idx < n) out[idx] = run;
        run += v[i];
    }
}

template <typename T>
static hipError_t scan_impl(const T* in, T* out, u64 n, T* tmp, hipStream_t s) {
    if (n == 0) return hipSuccess;
    u64 blocks = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(scan_reduce<T>, dim3((u32)blocks), dim3(kBlock), 0, s, in, n, tmp);
    hipLaunchKernelGGL(scan_single<T>, dim3(1), dim3(1024), 0, s, tmp, blocks);
    hipLaunchKernelGGL(scan_down<T>, dim3((u32)blocks), dim3(kBlock), 0, s, in, out, n, (const T*)tmp);
    return hipGetLastError();
}

hipError_t launch_scan_u32(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* tmp, hipStream_t s) {
    return scan_impl<u32>(in, out, n, tmp, s);
}
hipError_t launch_scan_u64(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* tmp, hipStream_t s) {
    return scan_impl<u64>((const u64*)in, (u64*)out, n, (u64*)tmp, s);
}

// ---------------------------------------------------------------------------
// run-length reduce of sorted spill keys (reduceKMers after a real sort)
// ---------------------------------------------------------------------------

template <int W>
__global__ __launch_bounds__(kBlock) void rle_heads(const u64* __restrict__ keys, u64 stride, u64 n,
                                                    u32* __restrict__ flags) {
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
        u32 h = 1;
        if (i > 0) {
            bool same = true;
#pragma unroll
            for (int j = 0; j < W; j++) same = same && keys[(u64)j * stride + i] == keys[(u64)j * stride + i - 1];
            h = same ? 0u : 1u;
        }
        flags[i] = h;
    }
}

template <int W>
__global__ __launch_bounds__(kBlock) void rle_scatter(const u64* __restrict__ keys, u64 stride, u64 n,
                                                      const u32* __restrict__ flags, const u32* __restrict__ pos,
                                                      u64* __restrict__ out, u64 ostride, u32* __restrict__ head) {
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
        if (!flags[i]) continue;
        u32 q = pos[i];
#pragma unroll
        for (int j = 0; j < W; j++) out[(u64)j * ostride + q] = keys[(u64)j * stride + i];
        head[q] = (u32)i;
    }
}

__global__ __launch_bounds__(kBlock) void rle_counts_k(const u32* __restrict__ head, u64 m, u64 n,
                                                       u32* __restrict__ cnts) {
    for (u64 q = (u64)blockIdx.x * kBlock + threadIdx.x; q < m; q += (u64)gridDim.x * kBlock) {
        u64 end = (q + 1 < m) ? (u64)head[q + 1] : n;
        cnts[q] = (u32)(end - head[q]);
    }
}

static int grid_for(u64 n, int cap = 8192) {
    u64 g = (n + kBlock - 1) / kBlock;
    if (g > (u64)cap) g = cap;
    return (int)(g ? g : 1);
}

hipError_t launch_rle_heads(int W, const uint64_t* keys, uint64_t stride, uint64_t n, uint32_t* flags,
                            hipStream_t s) {
    int g = grid_for(n);
    switch (W) {
    case 1: hipLaunchKernelGGL(rle_heads<1>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, flags); break;
    case 2: hipLaunchKernelGGL(rle_heads<2>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, flags); break;
    case 3: hipLaunchKernelGGL(rle_heads<3>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, flags); break;
    case 4: hipLaunchKernelGGL(rle_heads<4>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, flags); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_rle_scatter(int W, const uint64_t* keys, uint64_t stride, uint64_t n, const uint32_t* flags,
                              const uint32_t* pos, uint64_t* out_keys, uint64_t out_stride, uint32_t* head_idx,
                              hipStream_t s) {
    int g = grid_for(n);
    switch (W) {
    case 1: hipLaunchKernelGGL(rle_scatter<1>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, flags, pos, out_keys, out_stride, head_idx); break;
    case 2: hipLaunchKernelGGL(rle_scatter<2>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, flags, pos, out_keys, out_stride, head_idx); break;
    case 3: hipLaunchKernelGGL(rle_scatter<3>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, flags, pos, out_keys, out_stride, head_idx); break;
    case 4: hipLaunchKernelGGL(rle_scatter<4>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, flags, pos, out_keys, out_stride, head_idx); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_rle_counts(const uint32_t* head_idx, uint64_t m, uint64_t n, uint32_t* cnts, hipStream_t s) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(rle_counts_k, dim3(grid_for(m)), dim3(kBlock), 0, s, head_idx, m, n, cnts);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// pack: SoA -> SortedKMerFile records (W LE u64 words + LE u32 count)
// ---------------------------------------------------------------------------

template <int W>
__global__ __launch_bounds__(kBlock) void pack_records(const u64* __restrict__ keys, u64 stride,
                                                       const u32* __restrict__ cnts, u64 n, u32* __restrict__ out) {
    constexpr int RW = 2 * W + 1;  // u32 words per record
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
        u32* o = out + i * RW;
#pragma unroll
        for (int j = 0; j < W; j++) {
            u64 v = keys[(u64)j * stride + i];
            o[2 * j] = (u32)v;
            o[2 * j + 1] = (u32)(v >> 32);
        }
        o[2 * W] = cnts[i];
    }
}

hipError_t launch_pack(int W, const uint64_t* keys, uint64_t stride, const uint32_t* cnts, uint64_t n, void* out,
                       hipStream_t s) {
    if (n == 0) return hipSuccess;
    int g = grid_for(n);
    switch (W) {
    case 1: hipLaunchKernelGGL(pack_records<1>, dim3(g), dim3(kBlock), 0, s, keys, stride, cnts, n, (u32*)out); break;
    case 2: hipLaunchKernelGGL(pack_records<2>, dim3(g), dim3(kBlock), 0, s, keys, stride, cnts, n, (u32*)out); break;
    case 3: hipLaunchKernelGGL(pack_records<3>, dim3(g), dim3(kBlock), 0, s, keys, stride, cnts, n, (u32*)out); break;
    case 4: hipLaunchKernelGGL(pack_records<4>, dim3(g), dim3(kBlock), 0, s, keys, stride, cnts, n, (u32*)out); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Partition engine, passes P4/P5: after P2 (scatter by hash digit 48..55) and
// P3 (stable radix pass by hash digit 56..63) the keys are grouped by bucket =
// hash >> 48. P4 finds every bucket's range by binary search; P5 counts each
// bucket in an LDS-resident open-addressed table (one 1024-thread workgroup
// per CU walks the buckets) and appends the bucket's distinct (key, count)
// records with one global reservation per bucket. Keys that do not fit the
// LDS table fall back to the global table (and from there to the spill
// buffer), so the count stays exact for any input.
// ---------------------------------------------------------------------------

template <int W>
__global__ __launch_bounds__(kBlock) void bucket_bounds_k(const u64* __restrict__ keys, u64 stride, u64 n, int bits,
                                                          u64* __restrict__ starts) {
    const u64 nb = 1ull << bits;
    for (u64 b = (u64)blockIdx.x * kBlock + threadIdx.x; b <= nb; b += (u64)gridDim.x * kBlock) {
        u64 lo = 0, hi = n;
        while (lo < hi) {
            u64 mid = (lo + hi) >> 1;
            const u64 k0 = keys[stride ? mid : mid * W];  // (stride 0: W consecutive words per key)
            if ((k0 >> (64 - bits)) < b)
                lo = mid + 1;
            else
                hi = mid;
        }
        starts[b] = lo;
    }
}

hipError_t launch_bucket_bounds(int W, const uint64_t* keys, uint64_t stride, uint64_t n, int bits, uint64_t* starts,
                                hipStream_t s) {
    u64 nb = (1ull << bits) + 1;
    int g = (int)((nb + kBlock - 1) / kBlock);
    switch (W) {
    case 1: hipLaunchKernelGGL(bucket_bounds_k<1>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, bits, starts); break;
    case 2: hipLaunchKernelGGL(bucket_bounds_k<2>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, bits, starts); break;
    case 3: hipLaunchKernelGGL(bucket_bounds_k<3>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, bits, starts); break;
    case 4: hipLaunchKernelGGL(bucket_bounds_k<4>, dim3(g), dim3(kBlock), 0, s, keys, stride, n, bits, starts); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

constexpr int kBucketBlock = 1024;
constexpr int kBucketWaves = kBucketBlock / 64;

// Exclusive scan across a workgroup of NT threads (NT/64 waves); lds holds
// NT/64 u32. Returns this thread's exclusive prefix; *total = block sum.
template <int NT>
__device__ __forceinline__ u32 block_excl_scan_n(u32 v, u32* lds, u32* total) {
    constexpr int NW = NT / 64;
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u32 x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        u32 y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wave] = x;
    __syncthreads();
    u32 before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        u32 t = lds[w];
        before += (w < wave) ? t : 0u;
        tot += t;
    }
    *total = tot;
    __syncthreads();
    return before + x - v;
}

int bucket_lds_slots(int W) {
    // slot: W key words + u32 count (+ u32 state for W >= 2); ~139 KiB per CU
    // (the rest: per-wave slow-path queues); multiple of 64, <= SegCfg CAP
    int per = 8 * W + 4 + (W >= 2 ? 4 : 0);
    int slots = (139 * 1024) / per;
    return slots / 64 * 64;
}

struct BucketArgs {
    const u64* keys;
    u64 stride;
    const u64* starts;
    u32 nbuckets;
    u32 lcap;
    u64* rec_keys;  // SoA, rec_cap stride
    u32* rec_cnts;
    u64 rec_cap;
    u64* rec_cursor;
    u64* table;
    u64 cap;
    u64* spill;
    u64 spill_cap;
    u64* spill_ctr;
    u64* stats;
    u32 probe_limit;
    u64* desc_key;    // segment descriptors: bucket << 48 | first key fraction of the pass
    u64* desc_start;  //   first record
    u32* desc_len;    //   records
    u64 desc_cap;
    int skip;         // timing experiments only (KC_P5_SKIP): 1 = no LDS inserts
    int distinct;     // input where most keys are distinct (high cardinality): a bucket's
                      // first split m is taken from its key count (no aborted first pass)
    const u64* sub_starts;  // pre-split buckets (high cardinality): 256 sub-buckets per bucket by key bits
                            // 40..47, sub_starts[b * 256 + d] (2^24 + 1 entries); nullptr: plain buckets
    const unsigned char* run_flags;     // pre-split, after sort_runs_k: only the runs it flagged
    const unsigned char* bucket_flags;  //   (run_flags[b * 256 + first sub-bucket], bucket_flags[b])
    u32 run_per;                        //   packed with sort_runs_k's run size (0: the table's)
};

// 48-bit slot fraction of a key for the P5 LDS table: multiply-shift (the
// high bits of key * odd constant depend on every key bit); the keys of one
// bucket share their top 16 bits, which the multiply spreads as well.
template <int W>
__device__ __forceinline__ u64 slot_frac(const u64 (&key)[W]) {
    u64 h = key[0] * 0x9e3779b97f4a7c15ull;
#pragma unroll
    for (int j = 1; j < W; j++) h = (h ^ (h >> 29)) + key[j] * 0xc2b2ae3d27d4eb4full;
    return h >> 16;
}

// LDS tables of one-word keys in groups of 4 slots (32 B, read as two 16-byte
// halves): logical slot j of group g sits at physical slot 4g + (j ^ gswz(g)),
// i.e. the two halves swap places in every other run of 8 groups. Unswizzled,
// a half's 16 bytes start at one of only 8 of the 16 four-bank quads (32-byte
// groups), so the 16 lanes of a ds_read_b128 lane group meet twice as often
// on a quad; swizzled, the halves of random groups spread over all 16.
#ifndef KC_NO_GSWZ
__device__ __forceinline__ u32 gswz(u32 g) { return (g >> 2) & 2u; }
#else
__device__ __forceinline__ u32 gswz(u32) { return 0u; }  // variant builds: the unswizzled layout (A/B)
#endif

// `frac` is a 48-bit uniform hash fraction; slot = frac * lcap >> 48.
// *claimed is set when this key took an empty slot.
template <int W, int GS = 4>
__device__ __forceinline__ bool lds_insert(const u64 (&key)[W], u64 frac, u64* lkeys, u32* lcnt, u32* lstate,
                                           u32 lcap, u32 max_probe, bool* claimed, u32 w = 1u) {
    static_assert(GS == 2 || GS == 4, "LDS group of 2 or 4 slots");
    u32 slot = (u32)((frac * (u64)lcap) >> 48);
    if constexpr (W == 1) {
        if ((lcap % GS) == 0) {
            // groups of GS slots: the home group is read with GS/2 16-byte LDS
            // loads and a repeat (the common case) resolves with branch-free
            // compares and one add; probing continues group by group
            const u32 ng = lcap / GS;
            u32 g = (u32)((frac * (u64)ng) >> 48);
            for (u32 pr = 0; pr < max_probe; pr += GS) {
                const u32 sw = GS == 4 ? gswz(g) : 0u;  // physical slot of logical j: GS g + (j ^ sw)
                u64 v[GS];
#pragma unroll
                for (int h = 0; h < GS / 2; h++) {
                    const v2u64 a = *(const lds_v2u64*)(lkeys + GS * g + ((2u * (u32)h) ^ sw));
                    v[2 * h] = a.x;
                    v[2 * h + 1] = a.y;
                }
                int hit = -1, emp = -1;
#pragma unroll
                for (int i = GS - 1; i >= 0; i--) {
                    if (v[i] == key[0]) hit = i;
                    if (v[i] == 0ull) emp = i;
                }
                if (hit >= 0 && (emp < 0 || hit < emp)) {
                    atomicAdd(&lcnt[GS * g + ((u32)hit ^ sw)], w);
                    return true;
                }
                if (emp >= 0) {
                    // claim the first empty slot; a lost race re-reads the group
                    const u64 old = atomicCAS((unsigned long long*)&lkeys[GS * g + ((u32)emp ^ sw)], 0ull,
                                              (unsigned long long)key[0]);
                    if (old == 0ull || old == key[0]) {
                        atomicAdd(&lcnt[GS * g + ((u32)emp ^ sw)], w);
                        *claimed = old == 0ull;
                        return true;
                    }
                    pr -= GS;  // same group again
                    continue;
                }
                if (++g == ng) g = 0;
            }
            return false;
        }
        for (u32 pr = 0; pr < max_probe; ++pr) {
            // read first: a repeat (the common case) costs a read and one add;
            // only an EMPTY reading is confirmed by the CAS
            u64 old = __hip_atomic_load(&lkeys[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old == 0ull) old = atomicCAS((unsigned long long*)&lkeys[slot], 0ull, (unsigned long long)key[0]);
            if (old == 0ull || old == key[0]) {
                atomicAdd(&lcnt[slot], w);
                *claimed = old == 0ull;
                return true;
            }
            if (++slot == lcap) slot = 0;
        }
        return false;
    } else {
        // as insert_wide: one attempt per iteration, no divergent spin
        u32 pr = 0;
        for (;;) {
            u32 st = __hip_atomic_load(&lstate[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (st == 0u) {
                u32 prev = atomicCAS(&lstate[slot], 0u, 1u);
                if (prev == 0u) {
#pragma unroll
                    for (int j = 0; j < W; j++) lkeys[(size_t)j * lcap + slot] = key[j];
                    atomicAdd(&lcnt[slot], w);
                    __hip_atomic_store(&lstate[slot], 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    *claimed = true;
                    return true;
                }
                st = prev;
            }
            if (st == 1u) continue;  // being published: retry the same slot
            bool eq = true;
#pragma unroll
            for (int j = 0; j < W; j++) eq = eq && lkeys[(size_t)j * lcap + slot] == key[j];
            if (eq) {
                atomicAdd(&lcnt[slot], w);
                return true;
            }
            if (++pr >= max_probe) return false;
            if (++slot == lcap) slot = 0;
        }
    }
}

// P5: one 1024-thread block per bucket at a time counts the bucket's keys in
// an LDS open-addressed table and emits (key, count) records. A bucket with
// more distinct keys than the table holds (high-cardinality input, SURVEY
// cfg5) is counted in m sub-range passes: pass j takes the keys whose hash
// fraction ((h & 2^48-1) * m) >> 48 equals j and slots them by the remaining
// fraction bits, so every pass uses the whole table. m starts at 1; a pass
// whose table passes ~81% fill aborts, the LDS table is cleared and m grows
// by a power of two (estimated from fill / keys scanned), so finished
// sub-ranges stay valid. Only at m == kMaxSub do keys that miss the table go
// to the global fallback table and then to the spill buffer.
constexpr u32 kMaxSub = 1024;
constexpr u32 kQueue = 128;  // P5 per-wave slow-path queue entries (u32)

template <int W>
__global__ __launch_bounds__(kBucketBlock) void count_buckets(BucketArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64* lkeys = (u64*)smem;                                  // W x lcap
    u32* lcnt = (u32*)(lkeys + (size_t)W * a.lcap);           // lcap
    u32* lstate = lcnt + a.lcap;                              // lcap (W >= 2)
    u32* misc = lstate + (W >= 2 ? a.lcap : 0);               // scan scratch (16), base (2), fill, abort, m
    u32* lfill = misc + 20;
    u32* labort = misc + 21;
    u32* lnext = misc + 22;
    u32* wtot_l = misc + 24;  // kBucketWaves per-wave record counts
    const int tid = threadIdx.x;
    const int lane = (int)lane_id();
    const u64 lane_lt = lanemask_lt();
    u32* wq = misc + 48 + (tid >> 6) * kQueue;  // this wave's slow-path queue (bucket offsets)
    for (u32 i = tid; i < a.lcap; i += kBucketBlock) {
#pragma unroll
        for (int j = 0; j < W; j++) lkeys[(size_t)j * a.lcap + i] = 0ull;
        lcnt[i] = 0;
        if constexpr (W >= 2) lstate[i] = 0;
    }
    if (tid == 0) {
        *lfill = 0;
        *labort = 0;
    }
    __syncthreads();
    const u32 limit = (a.lcap * 13u) >> 4;
    const u32 mmax = a.lcap >= 64 ? kMaxSub : 1u;  // tiny test tables: global fallback only
    for (u32 b = blockIdx.x; b < a.nbuckets; b += gridDim.x) {
        if (a.bucket_flags && !a.bucket_flags[b]) continue;  // block-uniform
        // a full record buffer ends the launch early (the host reruns P5)
        if (tid == 0)
            *lnext = (u32)(__hip_atomic_load((unsigned long long*)&a.stats[ST_ERR], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) &
                           ERR_REC_OVERFLOW);
        __syncthreads();
        const bool stop = uni32(*lnext) != 0u;
        __syncthreads();
        if (stop) return;
        // Pre-split buckets: runs of consecutive sub-buckets holding at most
        // `per` keys are counted in one pass each (distinct <= keys: the
        // table never fills, every key is read once); a sub-bucket with more
        // keys is split by the bits below it (fshift = 40) as plain buckets
        // are by the bits below the bucket (fshift = 48).
        const u64 per = a.run_per ? (u64)a.run_per : (u64)limit * 7 / 8;
        u32 sb = 0;
        bool once = false;
        for (;;) {
        u64 lo, hi;
        u32 fshift = 48;
        bool multi = false;
        u32 nsub_l2 = 0;  // multi: ceil(log2(sub-buckets in the run))
        u64 dbase = (u64)b << 48;
        if (a.sub_starts) {
            if (sb >= 256u) break;
            const u64* ss = a.sub_starts + (u64)b * 256u;
            const u32 s0 = sb;
            lo = ss[s0];
            u32 e = s0 + 1;
            while (e < 256u && ss[e + 1] - lo <= per) e++;
            hi = ss[e];
            sb = e;
            multi = hi - lo <= per;
            fshift = multi ? 48u : 40u;
            while ((1u << nsub_l2) < e - s0) nsub_l2++;
            dbase |= (u64)s0 << 40;
            if (hi == lo) continue;
            if (a.run_flags && !a.run_flags[(u64)b * 256u + s0]) continue;  // sorted by sort_runs_k
        } else {
            if (once) break;
            once = true;
            lo = a.starts[b];
            hi = a.starts[b + 1];
            if (hi == lo) continue;
        }
        const u64 FM = (1ull << fshift) - 1;
        u32 m = 1, sub = 0;
        if (a.distinct && !multi) {
            // every key may be distinct: enough passes that each fills the
            // table to at most 7/8 of its abort limit
            while (m < mmax && (u64)m * per < hi - lo) m *= 2;
        }
        while (sub < m) {
            const bool last = m >= mmax || multi;
            u64 scanned = 0;
            u32 qn = 0;  // entries in this wave's queue (wave-uniform)
            // slow path for the first c queued keys: full probing insert, fill
            // and abort accounting, last-resort global table and spill
            auto drain = [&](u32 c) {
                const bool act = lane < (int)c;
                u64 qk[W];
#pragma unroll
                for (int j = 0; j < W; j++) qk[j] = 0;
                if (act) {
                    const u64 gi = lo + wq[lane];
                    load_key<W>(a.keys, a.stride, gi, qk);
                }
                bool done = true, claimed = false, lclaim = false, full = false;
                if (act) {
                    if (!lds_insert<W>(qk, slot_frac<W>(qk), lkeys, lcnt, lstate, a.lcap,
                                       last ? a.lcap : (a.lcap < 64u ? a.lcap : 64u), &lclaim)) {
                        if (!last) {
                            full = true;
                        } else if constexpr (W == 1) {
                            done = insert_w1(qk[0], a.table, a.cap, a.probe_limit, &claimed);
                        } else {
                            done = insert_wide<W>(qk, a.table, a.cap, a.probe_limit, &claimed);
                        }
                    }
                }
                const u64 lm = __ballot(lclaim);
                const u64 fm = __ballot(full);
                if (!last && (lm || fm) && lane == 0) {
                    u32 f = atomicAdd(lfill, (u32)__popcll(lm)) + (u32)__popcll(lm);
                    if (fm || f > limit) atomicOr(labort, 1u);
                }
                if (last) {
                    u64 cm = __ballot(claimed);
                    if (cm && lane == __ffsll((long long)cm) - 1)
                        atomicAdd((unsigned long long*)&a.stats[ST_CLAIMED], (unsigned long long)__popcll(cm));
                    bool spill = !done;
                    if (__ballot(spill)) {
                        u64 idx = wave_reserve(a.spill_ctr, spill);
                        if (spill) {
                            if (idx < a.spill_cap) {
#pragma unroll
                                for (int j = 0; j < W; j++) a.spill[(u64)j * a.spill_cap + idx] = qk[j];
                            } else {
                                atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_SPILL_OVERFLOW);
                            }
                        }
                    }
                }
            };
            constexpr int U = (W == 1) ? 8 : 4;  // independent key loads in flight per thread
            // software pipeline: the next iteration's keys are loaded before
            // this iteration's inserts, so HBM latency overlaps LDS work
            u64 nkey[U][W];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const u64 i = lo + (u64)u * kBucketBlock + tid;
                load_key<W>(a.keys, a.stride, min(i, hi - 1), nkey[u]);
            }
            for (u64 base = lo; base < hi; base += (u64)U * kBucketBlock) {
                if (!last && __hip_atomic_load(labort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                scanned += (u64)U * kBucketBlock;
                u64 key[U][W];
                bool live[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const u64 i = base + (u64)u * kBucketBlock + tid;
                    live[u] = i < hi;
#pragma unroll
                    for (int j = 0; j < W; j++) key[u][j] = nkey[u][j];
                }
                const u64 nbase = base + (u64)U * kBucketBlock;
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const u64 i = nbase + (u64)u * kBucketBlock + tid;
                    load_key<W>(a.keys, a.stride, min(i, hi - 1), nkey[u]);
                }
                // fast path, branch-light: a key already in its home group (W=1)
                // or home slot (W>=2) is counted in place; every other wanted
                // key goes to the wave's queue (its offset in the bucket), and
                // the queue is drained 64 keys at a time with all lanes active
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const u64 gi = base + (u64)u * kBucketBlock + tid;
                    const bool want =
                        live[u] && !a.skip && (u32)(((key[u][0] & FM) * (u64)m) >> fshift) == sub;
                    bool found = false;
                    const u64 fr = slot_frac<W>(key[u]);
                    if (multi) {
                        // a run of sub-buckets (<= per keys, mostly distinct):
                        // insert in place with full probing; the queue keeps
                        // only what misses the table (none while keys <= per)
                        bool lclaim = false;
                        found = want && lds_insert<W>(key[u], fr, lkeys, lcnt, lstate, a.lcap, a.lcap, &lclaim);
                    } else if constexpr (W == 1) {
                        if ((a.lcap & 3u) == 0) {
                            const u32 g = (u32)((fr * (u64)(a.lcap >> 2)) >> 48);
                            const u32 sw = gswz(g);
                            const v2u64 a0 = *(const lds_v2u64*)(lkeys + 4 * g + sw);
                            const v2u64 a1 = *(const lds_v2u64*)(lkeys + 4 * g + (2u ^ sw));
                            const u64 v[4] = {a0.x, a0.y, a1.x, a1.y};
                            int hit = -1, emp = -1;
#pragma unroll
                            for (int i = 3; i >= 0; i--) {
                                if (v[i] == key[u][0]) hit = i;
                                if (v[i] == 0ull) emp = i;
                            }
                            found = want && hit >= 0 && (emp < 0 || hit < emp);
                            if (found) atomicAdd(&lcnt[4 * g + ((u32)hit ^ sw)], 1u);
                        }
                    } else {
                        const u32 sl = (u32)((fr * (u64)a.lcap) >> 48);
                        if (__hip_atomic_load(&lstate[sl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 2u) {
                            bool eq = true;
#pragma unroll
                            for (int j = 0; j < W; j++) eq = eq && lkeys[(size_t)j * a.lcap + sl] == key[u][j];
                            found = want && eq;
                            if (found) atomicAdd(&lcnt[sl], 1u);
                        }
                    }
                    const bool pend = want && !found;
                    const u64 pb = __ballot(pend);
                    if (pb) {
                        if (pend) wq[qn + (u32)__popcll(pb & lane_lt)] = (u32)(gi - lo);
                        qn += (u32)__popcll(pb);
                        if (qn >= 64) {
                            drain(64);
                            // keep the overflow (< 64 entries) at the queue front
                            const u32 rest = qn - 64;
                            const u32 keep = lane < (int)rest ? wq[64 + lane] : 0u;
                            if (lane < (int)rest) wq[lane] = keep;
                            qn = rest;
                        }
                    }
                }
            }
            // leftovers (an aborted pass is restarted from scratch instead)
            if (qn && (last || !__hip_atomic_load(labort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) drain(qn);
            __syncthreads();
            const bool aborted = uni32(*labort) != 0u;  // every thread reads before tid 0 resets it
            __syncthreads();
            if (aborted) {
                // finer split: m' = m * 2^s from the fill rate seen so far
                if (tid == 0) {
                    const u64 est = (u64)(*lfill) * m * (hi - lo) / (scanned ? scanned : 1);
                    u32 nm = m * 2;
                    while (nm < mmax && (u64)nm * ((u64)limit * 7 / 8) < est) nm *= 2;
                    *lnext = nm < mmax ? nm : mmax;
                    *lfill = 0;
                    *labort = 0;
                    atomicAdd((unsigned long long*)&a.stats[ST_P5_ABORTS], 1ull);
                    atomicMax((unsigned long long*)&a.stats[ST_P5_MAXM], (unsigned long long)*lnext);
                }
                for (u32 i = tid; i < a.lcap; i += kBucketBlock) {
#pragma unroll
                    for (int j = 0; j < W; j++) lkeys[(size_t)j * a.lcap + i] = 0ull;
                    lcnt[i] = 0;
                    if constexpr (W >= 2) lstate[i] = 0;
                }
                __syncthreads();
                const u32 nm = uni32(*lnext);
                sub *= nm / m;
                m = nm;
                __syncthreads();
                continue;
            }
            // emit the occupied slots: wave w owns slots [w*spw, (w+1)*spw);
            // it counts them with ballots, one 16-entry prefix gives its
            // output offset, and it writes its records in slot order (no
            // block-wide scans, two barriers per pass)
            {
                const int wave = tid >> 6;
                const u32 spw = (a.lcap + kBucketWaves - 1) / kBucketWaves;
                const u32 s0 = (u32)wave * spw;
                const u32 s1 = min(a.lcap, s0 + spw);
                u32 wc = 0;
                for (u32 c0 = s0; c0 < s1; c0 += 64) {
                    const u32 i = c0 + (u32)lane;
                    const bool occ = i < s1 && ((W == 1) ? (lkeys[i] != 0ull) : (lstate[i] == 2u));
                    wc += (u32)__popcll(__ballot(occ));
                }
                if (lane == 0) wtot_l[wave] = wc;
                __syncthreads();
                u32 total = 0, before = 0;
                for (int w = 0; w < kBucketWaves; w++) {
                    const u32 v = wtot_l[w];
                    before += w < wave ? v : 0u;
                    total += v;
                }
                if (tid == 0) {
                    u64 rbase = total ? atomicAdd((unsigned long long*)a.rec_cursor, (unsigned long long)total) : 0ull;
                    *(u64*)(misc + 16) = rbase;
                    if (rbase + total > a.rec_cap)
                        atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_REC_OVERFLOW);
                    *lfill = 0;
                    atomicAdd((unsigned long long*)&a.stats[ST_P5_PASSES], 1ull);
                    if (total) {
                        // the pass's records are the keys of bucket b whose next
                        // log2(m) bits equal sub: one key-ordered segment
                        const u64 di = atomicAdd((unsigned long long*)&a.stats[ST_DESC_FILL], 1ull);
                        if (di < a.desc_cap) {
                            // segment: the keys of [dbase, ...) whose next log2(m)
                            // bits below fshift equal sub (a run of sub-buckets:
                            // [dbase, dbase + run << 40)); len | the segment
                            // sort's digit shift << 24: digit = (key bits below
                            // 48 - the descriptor's) >> shift spans the 4096 bins
                            a.desc_key[di] = dbase | ((u64)sub << (fshift - __builtin_ctz(m)));
                            a.desc_start[di] = rbase;
                            const u32 dsh = multi ? 28u + nsub_l2 : fshift - 12u - (u32)__builtin_ctz(m);
                            a.desc_len[di] = total | (dsh << 24);
                        }
                    }
                }
                __syncthreads();
                u64 pos = *(u64*)(misc + 16) + before;
                const u64 lt = lanemask_lt();
                for (u32 c0 = s0; c0 < s1; c0 += 64) {
                    const u32 i = c0 + (u32)lane;
                    const bool occ = i < s1 && ((W == 1) ? (lkeys[i] != 0ull) : (lstate[i] == 2u));
                    const u64 bm = __ballot(occ);
                    if (occ) {
                        const u64 q = pos + (u64)__popcll(bm & lt);
                        if (q < a.rec_cap) {
#pragma unroll
                            for (int j = 0; j < W; j++)
                                a.rec_keys[(u64)j * a.rec_cap + q] = lkeys[(size_t)j * a.lcap + i];
                            a.rec_cnts[q] = lcnt[i];
                        }
                        // leave the slot empty for the next pass
#pragma unroll
                        for (int j = 0; j < W; j++) lkeys[(size_t)j * a.lcap + i] = 0ull;
                        lcnt[i] = 0;
                        if constexpr (W >= 2) lstate[i] = 0;
                    }
                    pos += (u64)__popcll(bm);
                }
            }
            __syncthreads();
            ++sub;
        }
        }
    }
}

// Sub-bucket starts of a pre-split partition: the regional radix pass over
// the 65536 buckets (regions) by key bits 40..47 wrote digit d of region r at
// pos[first tile of r][d], so sub-bucket r * 256 + d starts there (an empty
// region's sub-buckets start at the region's start).
__global__ __launch_bounds__(kBlock) void sub_starts_k(const u64* __restrict__ rstart, const u64* __restrict__ tpre,
                                                       const u64* __restrict__ pos, u32 nreg, u64 n,
                                                       u64* __restrict__ sub) {
    const u64 total = (u64)nreg * 256u;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i <= total; i += (u64)gridDim.x * kBlock) {
        if (i == total) {
            sub[i] = n;
            continue;
        }
        const u32 r = (u32)(i >> 8), d = (u32)(i & 255u);
        sub[i] = tpre[r + 1] > tpre[r] ? pos[tpre[r] * 256u + d] : rstart[r];
    }
}

hipError_t launch_sub_starts(const uint64_t* rstart, const uint64_t* tpre, const uint64_t* pos, uint32_t nreg,
                             uint64_t n, uint64_t* sub, hipStream_t s) {
    const u64 total = (u64)nreg * 256u + 1;
    hipLaunchKernelGGL(sub_starts_k, dim3(grid_for(total)), dim3(kBlock), 0, s, rstart, tpre, pos, nreg, n, sub);
    return hipGetLastError();
}

// P5s — pre-split buckets (high cardinality, after P3b): every run of
// consecutive sub-buckets holding at most SP keys is sorted in LDS and
// run-length encoded into sorted (key, count) records, one key-ordered segment
// per run (its descriptor flagged sorted: the finish copies it instead of
// sorting). The keys of a run lie in [b << 48 | s0 << 40, + (e - s0) << 40):
// an 11-bit digit over that span bins them (a counting pass and a scatter
// into LDS), each thread insertion-sorts its 2 bins, equal keys end up
// adjacent. A run holding one sub-bucket of more than SP keys, or a bin of
// more than kMaxSortBin keys (clustered keys), is flagged for the LDS hash
// table path (count_buckets over the flagged runs only).
// 512-thread workgroups, two per CU (LDS ~75 KB and <= 128 VGPRs each): one
// workgroup's loads and stores overlap the other's LDS sort (one 1024-thread
// workgroup per CU left every run's load latency and store drain exposed)
constexpr int kSrBlock = 512;
constexpr int kSrWaves = kSrBlock / 64;
constexpr u32 kSrBins = 2048;
constexpr u32 kSrBpt = kSrBins / kSrBlock;  // bins per thread in the bin scan
constexpr u32 kMaxSortBin = 48;

template <int W>
struct SortRunCfg {
    static constexpr int SP = W == 1 ? 8192 : (W == 2 ? 4096 : (W == 3 ? 2688 : 2048));  // keys per run
    static constexpr int R = (SP + kSrBlock - 1) / kSrBlock;                             // keys per thread
};

int sort_runs_keys(int W) { return W == 1 ? 8192 : (W == 2 ? 4096 : (W == 3 ? 2688 : 2048)); }

size_t sort_runs_lds(int W) {
    return (size_t)sort_runs_keys(W) * 8 * W + kSrBins * 4 + 64 * 4 + 257 * 8;
}

struct SortRunArgs {
    const u64* keys;
    u64 stride;
    const u64* sub_starts;  // 256 per bucket + 1
    u32 nbuckets;
    u64* rec_keys;
    u32* rec_cnts;
    u64 rec_cap;
    u64* rec_cursor;
    u64* stats;
    u64* desc_key;
    u64* desc_start;
    u32* desc_len;
    u64 desc_cap;
    unsigned char* run_flags;     // nbuckets * 256
    unsigned char* bucket_flags;  // nbuckets
    u32* nflag;                   // runs flagged
    u32* packed;                  // direct mode: SortedKMerFile records at pk_base + (run's first key) + rank
    u64 pk_base;
};

// one SortedKMerFile record (W LE u64 words + LE u32 count) at index pos
template <int W>
__device__ __forceinline__ void put_packed(u32* __restrict__ packed, u64 pos, const u64 (&k)[W], u32 cnt) {
    u32* o = packed + pos * (2 * W + 1);
#pragma unroll
    for (int j = 0; j < W; j++) {
        o[2 * j] = (u32)k[j];
        o[2 * j + 1] = (u32)(k[j] >> 32);
    }
    o[2 * W] = cnt;
}

template <int W>
__global__ __launch_bounds__(kSrBlock) __attribute__((amdgpu_waves_per_eu(4))) void sort_runs_k(SortRunArgs a) {
    constexpr int SP = SortRunCfg<W>::SP;
    constexpr int R = SortRunCfg<W>::R;
    constexpr u64 M48 = 0xffffffffffffull;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64* skey = (u64*)smem;                      // W x SP
    u32* bins = (u32*)(skey + (size_t)W * SP);   // kSrBins
    u32* misc = bins + kSrBins;                  // [0] flag, [1..16] wave sums, [20..21] record base
    u64* ss = (u64*)(misc + 64);                 // the bucket's 257 sub-bucket starts
    const int tid = threadIdx.x, lane = (int)lane_id(), wave = tid >> 6;
#ifdef KC_EXPERIMENTS
    // KC_EXPERIMENTS builds: block 0 prints its cycles per phase at the end
    u64 ph[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    u64 tl = wall_clock64();
#define SR_MARK(i)                         \
    do {                                   \
        const u64 tn = wall_clock64();     \
        ph[i] += tn - tl;                  \
        tl = tn;                           \
    } while (0)
#else
#define SR_MARK(i) \
    do {           \
    } while (0)
#endif
    for (u32 b = blockIdx.x; b < a.nbuckets; b += gridDim.x) {
        __syncthreads();
        if (tid <= 256) ss[tid] = a.sub_starts[(u64)b * 256u + tid];
        __syncthreads();
        u32 sb = 0;
        while (sb < 256u) {
            const u32 s0 = sb;
            const u64 lo = uni64(ss[s0]);
            // run end: the last e in [s0 + 1, 256] with ss[e] - lo <= SP (at
            // least s0 + 1) — count_buckets' greedy walk, by bisection
            u32 e = s0 + 1;
            {
                u32 eh = 256u;
                while (e < eh) {
                    const u32 mid = (e + eh + 1) >> 1;
                    if (le64_32(uni64(ss[mid]) - lo, (u32)SP))
                        e = mid;
                    else
                        eh = mid - 1;
                }
            }
            const u64 hi = uni64(ss[e]);
            sb = e;
            const u32 len = le64_32(hi - lo, (u32)SP) ? (u32)(hi - lo) : (u32)SP + 1u;
            SR_MARK(0);
            if (len == 0) continue;
            if (len > (u32)SP) {  // one sub-bucket of more than SP keys: hash path
                if (tid == 0) {
                    a.run_flags[(u64)b * 256u + s0] = 1;
                    a.bucket_flags[b] = 1;
                    atomicAdd(a.nflag, 1u);
                }
                continue;
            }
            // keys p = tid + i * kSrBlock (coalesced); positions past the run
            // load its last key (unconditional loads: no per-element waits)
            u64 k[R][W];
#pragma unroll
            for (int i = 0; i < R; i++) {
                const u32 p = min((u32)tid + (u32)i * kSrBlock, len - 1);
                load_key<W>(a.keys, a.stride, lo + p, k[i]);
            }
            u32 l2 = 0;
            while ((1u << l2) < e - s0) l2++;
            const int sh = 29 + (int)l2;  // (the descriptor's digit span: (e - s0) << 40 rounded up to 2^l2)
            const u64 base = (u64)s0 << 40;
            // bins over the run's exact span of e - s0 sub-buckets: digit =
            // floor(off / 2^29 * ceil(2^32 / span) / 2^32), monotone in the key
            // and < 2^11 (clamped); a span rounded up to a power of two would
            // leave up to half the bins empty and put twice the keys in the
            // others (bins over 8 keys take the slow position loop)
            const u32 span = e - s0;
            const u32 smul = (u32)((0x100000000ull + span - 1) / span);
            for (u32 i = tid; i < kSrBins; i += kSrBlock) bins[i] = 0;
            if (tid == 0) {
                misc[0] = 0;
                misc[23] = 0;
            }
            __syncthreads();
            SR_MARK(1);
            u32 dg[R];
#pragma unroll
            for (int i = 0; i < R; i++) {
                dg[i] = min((u32)(((u64)(u32)(((k[i][0] & M48) - base) >> 29) * smul) >> 32), kSrBins - 1);
                if ((u32)tid + (u32)i * kSrBlock < len) atomicAdd(&bins[dg[i]], 1u);
            }
            __syncthreads();
            SR_MARK(2);
            // bin starts: kSrBpt bins per thread, block-wide exclusive scan
            u32 cb[kSrBpt];
            u32 sum = 0, cmax = 0;
#pragma unroll
            for (u32 x = 0; x < kSrBpt; x++) {
                cb[x] = bins[kSrBpt * tid + x];
                sum += cb[x];
                cmax = max(cmax, cb[x]);
            }
            u32 inc = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const u32 y = __shfl_up(inc, o);
                if (lane >= o) inc += y;
            }
            if (lane == 63) misc[1 + wave] = inc;
            if (cmax > kMaxSortBin) misc[0] = 1u;
            __syncthreads();
            if (uni32(misc[0])) {  // clustered keys: hash path
                if (tid == 0) {
                    a.run_flags[(u64)b * 256u + s0] = 1;
                    a.bucket_flags[b] = 1;
                    atomicAdd(a.nflag, 1u);
                }
                __syncthreads();
                continue;
            }
            u32 wpre = 0;
            for (int w = 0; w < wave; w++) wpre += misc[1 + w];
            u32 bs = wpre + inc - sum;
#pragma unroll
            for (u32 x = 0; x < kSrBpt; x++) {
                bins[kSrBpt * tid + x] = bs;
                bs += cb[x];
            }
            __syncthreads();
            SR_MARK(3);
            u32 qs[R];  // each key's LDS slot (ties between equal keys)
#pragma unroll
            for (int i = 0; i < R; i++) {
                qs[i] = 0;
                if ((u32)tid + (u32)i * kSrBlock >= len) continue;
                const u32 q = atomicAdd(&bins[dg[i]], 1u);
                qs[i] = q;
#pragma unroll
                for (int j = 0; j < W; j++) skey[(size_t)j * SP + q] = k[i][j];
            }
            __syncthreads();
            SR_MARK(4);
            // each key's sorted position: its bin's start (bins now hold bin
            // ends) + the bin's smaller keys + the equal keys in earlier slots
            u32 pos[R];
            bool dup = false;
#pragma unroll
            for (int i = 0; i < R; i++) {
                const bool valid = (u32)tid + (u32)i * kSrBlock < len;
                const u32 d = dg[i];
                const u32 b0 = d ? bins[d - 1] : 0u, b1 = bins[d];
                const u32 nbn = valid ? b1 - b0 : 0u;
                // common case: word 0 against up to 8 bin entries read at
                // once (clamped, masked); ties or bigger bins take the loop
                constexpr int U8 = 8;
                u64 w0[U8];
#pragma unroll
                for (int x = 0; x < U8; x++) w0[x] = skey[min(b0 + (u32)x, (u32)SP - 1)];
                u32 r = b0;
                bool slow = nbn > (u32)U8;
#pragma unroll
                for (int x = 0; x < U8; x++) {
                    const bool in = (u32)x < nbn;
                    r += (in && w0[x] < k[i][0]) ? 1u : 0u;
                    slow |= in && w0[x] == k[i][0] && b0 + (u32)x != qs[i];
                }
                pos[i] = r;
                if (!slow) continue;
                r = b0;
                for (u32 x = b0; x < b1; x++) {
                    int c = 0;  // key x vs this key: -1 less, 0 equal, 1 greater
#pragma unroll
                    for (int jj = 0; jj < W; jj++) {
                        const u64 kx = skey[(size_t)jj * SP + x];
                        if (c == 0 && kx != k[i][jj]) c = kx < k[i][jj] ? -1 : 1;
                    }
                    r += (c < 0 || (c == 0 && x < qs[i])) ? 1u : 0u;
                    dup |= c == 0 && x != qs[i];
                }
                pos[i] = r;
            }
            if (dup) misc[23] = 1u;
            __syncthreads();
            SR_MARK(5);
            if (!uni32(misc[23]) && a.packed) {
                // direct mode, distinct keys: the run's records are its keys,
                // each written to its place in the finished packed run (the
                // run starts at its first key's position: no reservation)
                const u64 rbase = a.pk_base + lo;
                if (tid == 0) {
                    atomicAdd((unsigned long long*)a.rec_cursor, (unsigned long long)len);
                    atomicAdd((unsigned long long*)&a.stats[ST_P5_PASSES], 1ull);
                    const u64 di = atomicAdd((unsigned long long*)&a.stats[ST_DESC_FILL], 1ull);
                    if (di < a.desc_cap) {
                        a.desc_key[di] = ((u64)b << 48) | base;
                        a.desc_start[di] = rbase;
                        a.desc_len[di] = len | ((u32)(sh + 1) << 24) | (1u << 31);
                    }
                }
                // the keys into sorted order in LDS (every thread is past its
                // reads of skey: the barrier above), then the run's records
                // written as consecutive dwords: one wave store covers 256
                // contiguous bytes instead of 64 scattered records
#pragma unroll
                for (int i = 0; i < R; i++) {
                    if ((u32)tid + (u32)i * kSrBlock >= len) continue;
#pragma unroll
                    for (int jj = 0; jj < W; jj++) skey[(size_t)jj * SP + pos[i]] = k[i][jj];
                }
                __syncthreads();
                constexpr u32 RW = 2 * W + 1;  // dwords per SortedKMerFile record
                u32* __restrict__ out = a.packed + rbase * RW;
                const u32 nd = len * RW;
                for (u32 u = (u32)tid; u < nd; u += kSrBlock) {
                    const u32 r = u / RW, w = u - r * RW;
                    u32 v = 1u;
                    if (w < 2 * W) {
                        const u64 x = skey[(size_t)(w >> 1) * SP + r];
                        v = (w & 1u) ? (u32)(x >> 32) : (u32)x;
                    }
                    out[u] = v;
                }
                SR_MARK(8);
                continue;
            }
            if (!uni32(misc[23])) {
                // distinct keys (the high-cardinality case): records are the
                // keys, each written straight to its sorted place, count 1
                if (tid == 0) {
                    const u64 rbase = atomicAdd((unsigned long long*)a.rec_cursor, (unsigned long long)len);
                    *(u64*)(misc + 20) = rbase;
                    if (rbase + len > a.rec_cap)
                        atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_REC_OVERFLOW);
                    atomicAdd((unsigned long long*)&a.stats[ST_P5_PASSES], 1ull);
                    const u64 di = atomicAdd((unsigned long long*)&a.stats[ST_DESC_FILL], 1ull);
                    if (di < a.desc_cap) {
                        a.desc_key[di] = ((u64)b << 48) | base;
                        a.desc_start[di] = rbase;
                        a.desc_len[di] = len | ((u32)(sh + 1) << 24) | (1u << 31);  // sorted
                    }
                }
                __syncthreads();
                SR_MARK(6);
                const u64 rbase = *(const u64*)(misc + 20);
#pragma unroll
                for (int i = 0; i < R; i++) {
                    if ((u32)tid + (u32)i * kSrBlock >= len) continue;
                    const u64 r = rbase + pos[i];
                    if (r < a.rec_cap) {
#pragma unroll
                        for (int jj = 0; jj < W; jj++) a.rec_keys[(u64)jj * a.rec_cap + r] = k[i][jj];
                        a.rec_cnts[r] = 1u;
                    }
                }
                SR_MARK(8);
                continue;
            }
            // equal keys: the keys are permuted into sorted order in LDS and
            // run-length encoded
#pragma unroll
            for (int i = 0; i < R; i++) {
                if ((u32)tid + (u32)i * kSrBlock >= len) continue;
#pragma unroll
                for (int jj = 0; jj < W; jj++) skey[(size_t)jj * SP + pos[i]] = k[i][jj];
            }
            __syncthreads();
            // heads (first of equal keys) in strided order; record rank = heads
            // before the position (per-i wave ballots, then a scan of the
            // R x 16 wave totals in position order by wave 0)
            bool head[R];
            u32 hb[R];
#pragma unroll
            for (int i = 0; i < R; i++) {
                const u32 p = (u32)tid + (u32)i * kSrBlock;
                bool h = p < len;
                if (h && p > 0) {
                    bool eq = true;
#pragma unroll
                    for (int jj = 0; jj < W; jj++) eq = eq && skey[(size_t)jj * SP + p] == skey[(size_t)jj * SP + p - 1];
                    h = !eq;
                }
                head[i] = h;
                const u64 bm = __ballot(h);
                hb[i] = (u32)__popcll(bm & lanemask_lt());
                if (lane == 0) bins[i * kSrWaves + wave] = (u32)__popcll(bm);  // bins are free after the sort
            }
            __syncthreads();
            if (wave == 0) {
                constexpr u32 NV = R * kSrWaves;  // <= 128: two per lane
                static_assert(NV <= 128, "wave totals");
                const u32 x0 = 2u * (u32)lane, x1 = x0 + 1;
                const u32 v0 = x0 < NV ? bins[x0] : 0u, v1 = x1 < NV ? bins[x1] : 0u;
                const u32 sum = v0 + v1;
                u32 inc = sum;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const u32 y = __shfl_up(inc, o);
                    if (lane >= o) inc += y;
                }
                const u32 ex = inc - sum;
                if (x0 < NV) bins[x0] = ex;
                if (x1 < NV) bins[x1] = ex + v0;
                const u32 run = __shfl(inc, 63);
                if (lane == 0) {
                    u64 rbase;
                    if (a.packed) {  // direct mode: the run's place; gaps are compacted later
                        rbase = a.pk_base + lo;
                        atomicAdd((unsigned long long*)a.rec_cursor, (unsigned long long)run);
                    } else {
                        rbase = atomicAdd((unsigned long long*)a.rec_cursor, (unsigned long long)run);
                        if (rbase + run > a.rec_cap)
                            atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_REC_OVERFLOW);
                    }
                    *(u64*)(misc + 20) = rbase;
                    atomicAdd((unsigned long long*)&a.stats[ST_P5_PASSES], 1ull);
                    const u64 di = atomicAdd((unsigned long long*)&a.stats[ST_DESC_FILL], 1ull);
                    if (di < a.desc_cap) {
                        a.desc_key[di] = ((u64)b << 48) | base;
                        a.desc_start[di] = rbase;
                        a.desc_len[di] = run | ((u32)(sh + 1) << 24) | (1u << 31);  // sorted
                    }
                }
            }
            __syncthreads();
            SR_MARK(7);
            const u64 rbase = *(const u64*)(misc + 20);
#pragma unroll
            for (int i = 0; i < R; i++) {
                if (!head[i]) continue;
                const u32 p = (u32)tid + (u32)i * kSrBlock;
                u32 q = p + 1;
                while (q < len) {
                    bool eq = true;
#pragma unroll
                    for (int jj = 0; jj < W; jj++) eq = eq && skey[(size_t)jj * SP + q] == skey[(size_t)jj * SP + p];
                    if (!eq) break;
                    q++;
                }
                const u64 r = rbase + bins[i * kSrWaves + wave] + hb[i];
                if (a.packed) {
                    u64 kk[W];
#pragma unroll
                    for (int jj = 0; jj < W; jj++) kk[jj] = skey[(size_t)jj * SP + p];
                    put_packed<W>(a.packed, r, kk, q - p);
                } else if (r < a.rec_cap) {
#pragma unroll
                    for (int jj = 0; jj < W; jj++) a.rec_keys[(u64)jj * a.rec_cap + r] = skey[(size_t)jj * SP + p];
                    a.rec_cnts[r] = q - p;
                }
            }
            __syncthreads();
            SR_MARK(8);
        }
    }
#ifdef KC_EXPERIMENTS
    if (blockIdx.x == 0 && tid == 0)
        printf("kc: sort_runs block 0 ticks (100 MHz): scan %llu load %llu hist %llu binscan %llu scatter %llu "
               "isort %llu heads %llu tid0 %llu write %llu\n",
               (unsigned long long)ph[0], (unsigned long long)ph[1], (unsigned long long)ph[2],
               (unsigned long long)ph[3], (unsigned long long)ph[4], (unsigned long long)ph[5],
               (unsigned long long)ph[6], (unsigned long long)ph[7], (unsigned long long)ph[8]);
#endif
#undef SR_MARK
}

hipError_t launch_sort_runs(int W, const uint64_t* keys, uint64_t stride, const uint64_t* sub_starts,
                            uint32_t nbuckets, uint64_t* rec_keys, uint32_t* rec_cnts, uint64_t rec_cap,
                            uint64_t* rec_cursor, uint64_t* stats, uint64_t* desc_key, uint64_t* desc_start,
                            uint32_t* desc_len, uint64_t desc_cap, uint8_t* run_flags, uint8_t* bucket_flags,
                            uint32_t* nflag, int grid, hipStream_t s, void* packed, uint64_t pk_base) {
    SortRunArgs a;
    a.packed = (u32*)packed;
    a.pk_base = pk_base;
    a.keys = keys;
    a.stride = stride;
    a.sub_starts = sub_starts;
    a.nbuckets = nbuckets;
    a.rec_keys = rec_keys;
    a.rec_cnts = rec_cnts;
    a.rec_cap = rec_cap;
    a.rec_cursor = rec_cursor;
    a.stats = stats;
    a.desc_key = desc_key;
    a.desc_start = desc_start;
    a.desc_len = desc_len;
    a.desc_cap = desc_cap;
    a.run_flags = run_flags;
    a.bucket_flags = bucket_flags;
    a.nflag = nflag;
    const size_t lds = (sort_runs_lds(W) + 15) & ~(size_t)15;
    switch (W) {
    case 1: hipLaunchKernelGGL(sort_runs_k<1>, dim3(grid), dim3(kSrBlock), lds, s, a); break;
    case 2: hipLaunchKernelGGL(sort_runs_k<2>, dim3(grid), dim3(kSrBlock), lds, s, a); break;
    case 3: hipLaunchKernelGGL(sort_runs_k<3>, dim3(grid), dim3(kSrBlock), lds, s, a); break;
    case 4: hipLaunchKernelGGL(sort_runs_k<4>, dim3(grid), dim3(kSrBlock), lds, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Compaction of a packed run written in place by sort_runs_k (direct mode)
// whose runs held equal keys: segment order[d] (start dstart, records
// dlen & 0xffffff) moves to out_off[d] (u32 copies, one block per segment).
__global__ __launch_bounds__(kBlock) void packed_seg_copy_k(const u32* __restrict__ src, u32* __restrict__ dst, int rw,
                                                            const u32* __restrict__ order,
                                                            const u64* __restrict__ dstart,
                                                            const u32* __restrict__ dlen,
                                                            const u64* __restrict__ out_off, u64 ndesc, u64 base) {
    for (u64 d = blockIdx.x; d < ndesc; d += gridDim.x) {
        const u32 o = order[d];
        const u64 st = dstart[o];
        const u32 len = dlen[o] & 0xffffffu;
        const u64 ob = base + out_off[d];
        const u32 nw = len * (u32)rw;
        for (u32 x = threadIdx.x; x < nw; x += kBlock) dst[ob * (u64)rw + x] = src[st * (u64)rw + x];
    }
}

hipError_t launch_packed_seg_copy(int W, const void* src, void* dst, const uint32_t* order, const uint64_t* dstart,
                                  const uint32_t* dlen, const uint64_t* out_off, uint64_t ndesc, uint64_t base,
                                  int grid, hipStream_t s) {
    if (ndesc == 0) return hipSuccess;
    hipLaunchKernelGGL(packed_seg_copy_k, dim3(grid), dim3(kBlock), 0, s, (const u32*)src, (u32*)dst, 2 * W + 1,
                       order, dstart, dlen, out_off, ndesc, base);
    return hipGetLastError();
}

size_t bucket_lds_bytes(int W) {
    size_t lcap = (size_t)bucket_lds_slots(W);
    return lcap * (8 * W + 4 + (W >= 2 ? 4 : 0)) + (48 + (size_t)kBucketWaves * kQueue) * 4 + 16;
}

hipError_t launch_count_buckets(int W, const uint64_t* keys, uint64_t stride, const uint64_t* starts,
                                uint32_t nbuckets, uint64_t* rec_keys, uint32_t* rec_cnts, uint64_t rec_cap,
                                uint64_t* rec_cursor, uint64_t* table, uint64_t cap, uint64_t* spill,
                                uint64_t spill_cap, uint64_t* stats, uint32_t probe_limit, uint32_t lcap, int grid,
                                uint64_t* desc_key, uint64_t* desc_start, uint32_t* desc_len, uint64_t desc_cap,
                                hipStream_t s, bool distinct, const uint64_t* sub_starts,
                                const uint8_t* run_flags, const uint8_t* bucket_flags, uint32_t run_per) {
    BucketArgs a;
    a.run_flags = run_flags;
    a.bucket_flags = bucket_flags;
    a.run_per = run_per;
    a.skip = experiment_knob("KC_P5_SKIP");
    a.distinct = distinct ? 1 : 0;
    a.sub_starts = sub_starts;
    a.desc_key = desc_key;
    a.desc_start = desc_start;
    a.desc_len = desc_len;
    a.desc_cap = desc_cap;
    a.keys = keys;
    a.stride = stride;
    a.starts = starts;
    a.nbuckets = nbuckets;
    a.lcap = (lcap == 0 || lcap > (u32)bucket_lds_slots(W)) ? (u32)bucket_lds_slots(W) : lcap;
    a.rec_keys = rec_keys;
    a.rec_cnts = rec_cnts;
    a.rec_cap = rec_cap;
    a.rec_cursor = rec_cursor;
    a.table = table;
    a.cap = cap;
    a.spill = spill;
    a.spill_cap = spill_cap;
    a.spill_ctr = stats + ST_SPILL2_FILL;
    a.stats = stats;
    a.probe_limit = probe_limit;
    size_t lds = (bucket_lds_bytes(W) + 15) & ~(size_t)15;
    switch (W) {
    case 1: hipLaunchKernelGGL(count_buckets<1>, dim3(grid), dim3(kBucketBlock), lds, s, a); break;
    case 2: hipLaunchKernelGGL(count_buckets<2>, dim3(grid), dim3(kBucketBlock), lds, s, a); break;
    case 3: hipLaunchKernelGGL(count_buckets<3>, dim3(grid), dim3(kBucketBlock), lds, s, a); break;
    case 4: hipLaunchKernelGGL(count_buckets<4>, dim3(grid), dim3(kBucketBlock), lds, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Segmented sum after a sort: out index of element i = pos[i] + head[i] - 1
// (pos = exclusive scan of head flags); out_cnt must be zeroed.
template <int W>
__global__ __launch_bounds__(kBlock) void reduce_add_k(const u64* __restrict__ keys, u64 stride,
                                                       const u32* __restrict__ cnts, u64 n,
                                                       const u32* __restrict__ flags, const u32* __restrict__ pos,
                                                       u64* __restrict__ out_keys, u64 ostride,
                                                       u32* __restrict__ out_cnts) {
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
        u32 q = pos[i] + flags[i] - 1u;
        if (flags[i]) {
#pragma unroll
            for (int j = 0; j < W; j++) out_keys[(u64)j * ostride + q] = keys[(u64)j * stride + i];
        }
        atomicAdd(&out_cnts[q], cnts[i]);
    }
}

hipError_t launch_reduce_add(int W, const uint64_t* keys, uint64_t stride, const uint32_t* cnts, uint64_t n,
                             const uint32_t* flags, const uint32_t* pos, uint64_t* out_keys, uint64_t ostride,
                             uint32_t* out_cnts, hipStream_t s) {
    int g = grid_for(n);
    switch (W) {
    case 1: hipLaunchKernelGGL(reduce_add_k<1>, dim3(g), dim3(kBlock), 0, s, keys, stride, cnts, n, flags, pos, out_keys, ostride, out_cnts); break;
    case 2: hipLaunchKernelGGL(reduce_add_k<2>, dim3(g), dim3(kBlock), 0, s, keys, stride, cnts, n, flags, pos, out_keys, ostride, out_cnts); break;
    case 3: hipLaunchKernelGGL(reduce_add_k<3>, dim3(g), dim3(kBlock), 0, s, keys, stride, cnts, n, flags, pos, out_keys, ostride, out_cnts); break;
    case 4: hipLaunchKernelGGL(reduce_add_k<4>, dim3(g), dim3(kBlock), 0, s, keys, stride, cnts, n, flags, pos, out_keys, ostride, out_cnts); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// P3, regional scatter. After P2 the keys sit in 256 regions by the low bucket
// byte (word0 bits 48..55). P3 cuts every region into tiles of its own (a tile
// never straddles two regions) and scatters each tile by the high byte (bits
// 56..63). Positions come from a digit-major scan of per-tile histograms over
// region-ordered tiles, which is exactly bucket start + offset, so the order
// inside a tile does not matter: ranks are plain LDS atomics (no ballots), and
// a tile of 16K keys (1024 threads) writes digit runs long enough to fill
// whole lines. The next tile's keys are prefetched into registers.
// tiles: region r holds tiles [tpre[r], tpre[r+1]); tile i of r starts at
// rstart[r] + i * TILE.
// ---------------------------------------------------------------------------

constexpr int kP3Block = 1024;

template <int W>
struct P3Cfg {
    // keys per thread: the same tiles as rp_scatter_k<W,false> (rp_tile), which
    // scatters P3 with these tiles' histograms
    static constexpr int KPT = (W == 1) ? 16 : (W == 2 ? 8 : (W == 3 ? 5 : 4));
    static constexpr int TILE = kP3Block * KPT;
};

int p3_tile(int W) { return kP3Block * ((W == 1) ? 16 : (W == 2 ? 8 : (W == 3 ? 5 : 4))); }

__device__ __forceinline__ void p3_tile_range(const u64* __restrict__ rstart, const u64* __restrict__ tpre, u64 t,
                                              int TILE, u64* lo, u64* hi) {
    int a = 0, b = 256;  // region r with tpre[r] <= t < tpre[r+1]
    while (b - a > 1) {
        const int mid = (a + b) >> 1;
        if (tpre[mid] <= t)
            a = mid;
        else
            b = mid;
    }
    const u64 st = rstart[a] + (t - tpre[a]) * (u64)TILE;
    *lo = st;
    *hi = min(st + (u64)TILE, rstart[a + 1]);
}

// P3 tile histograms from the digit bytes P2 wrote (1 B per key instead of
// re-reading 8W B keys): 256-thread blocks, one private histogram per wave,
// 16 digits per thread per load (uint4 of bytes, tile-aligned)
template <int W>
__global__ __launch_bounds__(kBlock) void p3_upsweep_k(const unsigned char* __restrict__ digs,
                                                       const u64* __restrict__ rstart, const u64* __restrict__ tpre,
                                                       u64 ntiles, u32* __restrict__ cnt_t) {
    constexpr int TILE = P3Cfg<W>::TILE;
    __shared__ u32 h[4 * 256];
    const int tid = threadIdx.x, wave = tid >> 6;
    for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        for (int i = tid; i < 4 * 256; i += kBlock) h[i] = 0;
        __syncthreads();
        u64 lo, hi;
        p3_tile_range(rstart, tpre, t, TILE, &lo, &hi);
        u32* hw = h + wave * 256;
        // head up to 16-byte alignment, aligned body, tail
        const u64 alo = min(hi, (lo + 15) & ~15ull);
        for (u64 i = lo + tid; i < alo; i += kBlock) atomicAdd(&hw[digs[i]], 1u);
        const u64 ahi = alo + ((hi - alo) & ~15ull);
        for (u64 i = alo + 16 * (u64)tid; i < ahi; i += 16 * (u64)kBlock) {
            const v4u v = __builtin_nontemporal_load((const v4u*)(digs + i));
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const u32 w = c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
                atomicAdd(&hw[w & 255u], 1u);
                atomicAdd(&hw[(w >> 8) & 255u], 1u);
                atomicAdd(&hw[(w >> 16) & 255u], 1u);
                atomicAdd(&hw[w >> 24], 1u);
            }
        }
        for (u64 i = ahi + tid; i < hi; i += kBlock) atomicAdd(&hw[digs[i]], 1u);
        __syncthreads();
        cnt_t[t * 256 + tid] = h[tid] + h[256 + tid] + h[512 + tid] + h[768 + tid];  // tile-major, coalesced
        __syncthreads();
    }
}

// Positions from the tile-major counts, digit-major order: pos[t][d] =
// sum_{d' < d} total(d') + sum_{t' < t} cnt[t'][d], in three streaming kernels
// over chunks of kP3Chunk tiles (rows of 256 counts are read coalesced).
constexpr int kP3Chunk = 64;

__global__ __launch_bounds__(256) void p3_chunk_sum_k(const u32* __restrict__ cnt_t, u64 ntiles, u64* __restrict__ csum) {
    const u64 c = blockIdx.x;
    const u64 t0 = c * kP3Chunk, t1 = min(ntiles, t0 + kP3Chunk);
    u64 sum = 0;
    for (u64 t = t0; t < t1; t++) sum += cnt_t[t * 256 + threadIdx.x];
    csum[c * 256 + threadIdx.x] = sum;
}

// one block per digit: exclusive scan of that digit's chunk sums (each thread
// a run of consecutive chunks); the digit total goes to dtot[d]
__global__ __launch_bounds__(256) void p3_chunk_scan_k(u64* __restrict__ csum, u64 nchunks, u64* __restrict__ dtot) {
    __shared__ u64 part[256];
    const int d = blockIdx.x, t = threadIdx.x;
    const u64 per = (nchunks + 255) / 256;
    const u64 c0 = min(nchunks, (u64)t * per), c1 = min(nchunks, c0 + per);
    u64 sum = 0;
    for (u64 c = c0; c < c1; c++) sum += csum[c * 256 + d];
    part[t] = sum;
    __syncthreads();
    if (t == 0) {
        u64 acc = 0;
        for (int i = 0; i < 256; i++) {
            const u64 v = part[i];
            part[i] = acc;
            acc += v;
        }
        dtot[d] = acc;
    }
    __syncthreads();
    u64 run = part[t];
    for (u64 c = c0; c < c1; c++) {
        const u64 v = csum[c * 256 + d];
        csum[c * 256 + d] = run;
        run += v;
    }
}

__global__ __launch_bounds__(256) void p3_digit_base_k(u64* __restrict__ dtot) {
    if (threadIdx.x == 0) {
        u64 acc = 0;
        for (int i = 0; i < 256; i++) {
            const u64 v = dtot[i];
            dtot[i] = acc;
            acc += v;
        }
    }
}

__global__ __launch_bounds__(256) void p3_chunk_pos_k(const u32* __restrict__ cnt_t, const u64* __restrict__ csum,
                                                      const u64* __restrict__ dbase, u64 ntiles, u64* __restrict__ pos) {
    const u64 c = blockIdx.x;
    const u64 t0 = c * kP3Chunk, t1 = min(ntiles, t0 + kP3Chunk);
    u64 run = dbase[threadIdx.x] + csum[c * 256 + threadIdx.x];
    for (u64 t = t0; t < t1; t++) {
        pos[t * 256 + threadIdx.x] = run;
        run += cnt_t[t * 256 + threadIdx.x];
    }
}

template <int W>
__global__ __launch_bounds__(kP3Block) void p3_scatter_k(const u64* __restrict__ kin, u64* __restrict__ kout,
                                                         u64 stride, const u64* __restrict__ rstart,
                                                         const u64* __restrict__ tpre, u64 ntiles,
                                                         const u64* __restrict__ pos) {
    constexpr int KPT = P3Cfg<W>::KPT;
    constexpr int TILE = P3Cfg<W>::TILE;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64* skey = (u64*)smem;                 // W x TILE
    u32* wc = (u32*)(skey + (size_t)W * TILE);   // 16 waves x 128 words: two u16 rank counters each
    unsigned short* woff = (unsigned short*)(wc + 16 * 128);  // 16 x 256 wave offsets inside a digit
    u32* dst = (u32*)(woff + 16 * 256);     // 256 digit starts in the tile
    u64* gpos = (u64*)(dst + 256);          // 256 global run starts
    u32* wsum = (u32*)(gpos + 256);         // 16 wave partial sums
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    u64 nk[KPT][W];
    auto load = [&](u64 t) {
        if (t >= ntiles) return;
        u64 lo = 0, hi = 0;
        p3_tile_range(rstart, tpre, t, TILE, &lo, &hi);
        // unconditional loads, clamped into the (never empty) tile
#pragma unroll
        for (int i = 0; i < KPT; i++) {
            const u64 q = min(lo + (u64)i * kP3Block + tid, hi - 1);
#pragma unroll
            for (int j = 0; j < W; j++) nk[i][j] = __builtin_nontemporal_load(kin + (u64)j * stride + q);
        }
    };
    load(blockIdx.x);
    for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        u64 lo, hi;
        p3_tile_range(rstart, tpre, t, TILE, &lo, &hi);
        const u32 len = (u32)(hi - lo);
        u64 key[KPT][W];
#pragma unroll
        for (int i = 0; i < KPT; i++)
#pragma unroll
            for (int j = 0; j < W; j++) key[i][j] = nk[i][j];
        for (int i = tid; i < 16 * 128; i += kP3Block) wc[i] = 0;
        if (tid < 256) gpos[tid] = pos[t * 256 + tid];
        __syncthreads();
        load(t + gridDim.x);  // next tile's keys fly while this one is ranked
        // ranks inside the wave's own counters (atomics only collide within
        // a wave); a (wave, digit) offset table then orders the waves
        u32 rank[KPT];
#pragma unroll
        for (int i = 0; i < KPT; i++) {
            const u32 q = (u32)i * kP3Block + (u32)tid;
            if (q < len) {
                const u32 d = (u32)(key[i][0] >> 56);
                const u32 sh = 16 * (d & 1);
                rank[i] = (atomicAdd(&wc[wave * 128 + (d >> 1)], 1u << sh) >> sh) & 0xffffu;
            }
        }
        __syncthreads();
        // per digit: wave offsets, digit total, then digit starts (waves 0..3)
        if (tid < 256) {
            u32 run = 0;
            for (int w = 0; w < 16; w++) {
                woff[w * 256 + tid] = (unsigned short)run;
                run += (wc[w * 128 + (tid >> 1)] >> (16 * (tid & 1))) & 0xffffu;
            }
            const u32 v = run;
            u32 inc = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const u32 y = __shfl_up(inc, o);
                if (lane >= o) inc += y;
            }
            if (lane == 63) wsum[wave] = inc;
            dst[tid] = inc - v;
        }
        __syncthreads();
        if (tid < 256) {
            u32 add = 0;
            for (int w = 0; w < wave; w++) add += wsum[w];
            dst[tid] += add;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < KPT; i++) {
            const u32 q = (u32)i * kP3Block + (u32)tid;
            if (q < len) {
                const u32 d = (u32)(key[i][0] >> 56);
                const u32 at = dst[d] + woff[wave * 256 + d] + rank[i];
#pragma unroll
                for (int j = 0; j < W; j++) skey[(size_t)j * TILE + at] = key[i][j];
            }
        }
        __syncthreads();
        for (u32 q = tid; q < len; q += kP3Block) {
            const u64 k0 = skey[q];
            const u32 d = (u32)(k0 >> 56);
            const u64 g = gpos[d] + (q - dst[d]);
            kout[g] = k0;
#pragma unroll
            for (int j = 1; j < W; j++) kout[(u64)j * stride + g] = skey[(size_t)j * TILE + q];
        }
        __syncthreads();
    }
}

size_t p3_scatter_lds(int W) {
    return (size_t)W * p3_tile(W) * 8 + 16 * 128 * 4 + 16 * 256 * 2 + 256 * 4 + 256 * 8 + 16 * 4 + 16;
}

hipError_t launch_p3_hist(int W, const uint8_t* digs, const uint64_t* rstart, const uint64_t* tpre, uint64_t ntiles,
                          uint64_t* pos, uint64_t* tmp, int grid, hipStream_t s) {
    if (ntiles == 0) return hipSuccess;
    // tmp: ntiles x 256 u32 tile counts + p3_chunks(ntiles) x 256 u64 chunk sums
    u32* cnt_t = (u32*)tmp;
    u64* csum = tmp + (ntiles * 256 + 1) / 2;
    const u64 nchunks = (ntiles + kP3Chunk - 1) / kP3Chunk;
    const int gu = (int)hmin(ntiles, (u64)grid * 4);
#define KC_P3U(WW) \
    hipLaunchKernelGGL(p3_upsweep_k<WW>, dim3(gu), dim3(kBlock), 0, s, (const unsigned char*)digs, rstart, tpre, ntiles, cnt_t)
    switch (W) {
    case 1: KC_P3U(1); break;
    case 2: KC_P3U(2); break;
    case 3: KC_P3U(3); break;
    case 4: KC_P3U(4); break;
    default: return hipErrorInvalidValue;
    }
#undef KC_P3U
    u64* dtot = csum + nchunks * 256;
    hipLaunchKernelGGL(p3_chunk_sum_k, dim3(nchunks), dim3(256), 0, s, (const u32*)cnt_t, ntiles, csum);
    hipLaunchKernelGGL(p3_chunk_scan_k, dim3(256), dim3(256), 0, s, csum, nchunks, dtot);
    hipLaunchKernelGGL(p3_digit_base_k, dim3(1), dim3(256), 0, s, dtot);
    hipLaunchKernelGGL(p3_chunk_pos_k, dim3(nchunks), dim3(256), 0, s, (const u32*)cnt_t, (const u64*)csum,
                       (const u64*)dtot, ntiles, pos);
    return hipGetLastError();
}

uint64_t p3_tmp_elems(uint64_t ntiles) {
    return (ntiles * 256 + 1) / 2 + ((ntiles + kP3Chunk - 1) / kP3Chunk) * 256 + 256 + 8;
}

hipError_t launch_p3_scatter(int W, const uint64_t* kin, uint64_t* kout, uint64_t stride, const uint64_t* rstart,
                             const uint64_t* tpre, uint64_t ntiles, const uint64_t* hist, int grid, hipStream_t s) {
    if (ntiles == 0) return hipSuccess;
    const int g = (int)hmin(ntiles, (u64)grid);
    const size_t lds = (p3_scatter_lds(W) + 15) & ~(size_t)15;
#define KC_P3S(WW)                                                                                              \
    hipLaunchKernelGGL(p3_scatter_k<WW>, dim3(g), dim3(kP3Block), lds, s, kin, kout, stride, rstart, tpre, ntiles, \
                       (const u64*)hist)
    switch (W) {
    case 1: KC_P3S(1); break;
    case 2: KC_P3S(2); break;
    case 3: KC_P3S(3); break;
    case 4: KC_P3S(4); break;
    }
#undef KC_P3S
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Finish of the partition engine without a global sort. Buckets are key
// prefixes and every P5 pass is a key sub-range of its bucket, so the records
// of each pass (a segment, <= one LDS table) sorted in place and laid out in
// descriptor order are the whole sorted run.
//   desc_prep : sorted descriptor order -> lengths in that order
//   seg_sort  : one 1024-thread block per segment: LSD radix over the bytes
//               that vary inside the segment, stable wave-private ranking (8
//               ballots), exchange through LDS; writes SoA records at the
//               segment's output offset (counts gathered by original index)
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void desc_prep_k(const u32* __restrict__ order, const u32* __restrict__ len,
                                                      u64 n, u64* __restrict__ lens_sorted) {
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock)
        lens_sorted[i] = len[order[i]] & 0xffffffu;
}

__global__ __launch_bounds__(kBlock) void iota_k(u32* out, u64 n) {
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) out[i] = (u32)i;
}

__global__ __launch_bounds__(kBlock) void key_digits_k(const u64* __restrict__ keys, u64 lo, u64 hi, int shift,
                                                       unsigned char* __restrict__ out) {
    for (u64 i = lo + (u64)blockIdx.x * kBlock + threadIdx.x; i < hi; i += (u64)gridDim.x * kBlock)
        out[i] = (unsigned char)(keys[i] >> shift);
}

hipError_t launch_key_digits(const uint64_t* keys, uint64_t lo, uint64_t hi, int shift, uint8_t* out, hipStream_t s) {
    if (hi <= lo) return hipSuccess;
    if (shift < 0 || shift > 56) return hipErrorInvalidValue;
    hipLaunchKernelGGL(key_digits_k, dim3(grid_for(hi - lo)), dim3(kBlock), 0, s, keys, lo, hi, shift, out);
    return hipGetLastError();
}

hipError_t launch_iota_u32(uint32_t* out, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(iota_k, dim3(grid_for(n)), dim3(kBlock), 0, s, out, n);
    return hipGetLastError();
}

// The finish's group descriptors from the group bounds: order[g] = g,
// len[g] = (starts[g + 1] - starts[g]) | tag << 24 (lengths clamped to 24 bits:
// a longer group is past seg_sort's capacity, which *longest tells the host),
// *longest = the longest group (zeroed by the caller)
__global__ __launch_bounds__(kBlock) void group_desc_k(const u64* __restrict__ starts, u64 ng, u32 tag,
                                                       u32* __restrict__ order, u32* __restrict__ len,
                                                       u64* __restrict__ longest) {
    for (u64 i0 = (u64)blockIdx.x * kBlock; i0 < ng; i0 += (u64)gridDim.x * kBlock) {
        const u64 g = i0 + threadIdx.x;
        u64 l = 0;
        if (g < ng) {
            l = starts[g + 1] - starts[g];
            order[g] = (u32)g;
            len[g] = (u32)min(l, (u64)0xffffffu) | (tag << 24);
        }
        for (int o = 32; o >= 1; o >>= 1) l = max(l, (u64)__shfl_xor((long long)l, o));
        if (lane_id() == 0 && l) atomicMax((unsigned long long*)longest, (unsigned long long)l);
    }
}

hipError_t launch_group_desc(const uint64_t* starts, uint64_t ng, uint32_t tag, uint32_t* order, uint32_t* len,
                             uint64_t* longest, hipStream_t s) {
    if (ng == 0 || tag > 255) return hipErrorInvalidValue;
    hipLaunchKernelGGL(group_desc_k, dim3(grid_for(ng)), dim3(kBlock), 0, s, starts, ng, tag, order, len, longest);
    return hipGetLastError();
}

hipError_t launch_desc_prep(const uint32_t* order, const uint32_t* len, uint64_t n, uint64_t* lens_sorted,
                            hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(desc_prep_k, dim3(grid_for(n)), dim3(kBlock), 0, s, order, len, n, lens_sorted);
    return hipGetLastError();
}

constexpr int kSegBlock = 1024;
constexpr u32 kMaxBin = 64;  // seg_sort MSD fast path: largest bin sorted by insertion
constexpr int kSegWaves = kSegBlock / 64;

template <int W>
struct SegCfg {
    static constexpr int CAP = (W == 1) ? 11840 : (W == 2 ? 6144 : (W == 3 ? 4480 : 3584));  // >= bucket_lds_slots
    static constexpr int ITEMS = (CAP + kSegBlock - 1) / kSegBlock;
};

size_t seg_sort_msd_lds(int W) {
    int cap = W == 1 ? 11840 : (W == 2 ? 6144 : (W == 3 ? 4480 : 3584));
    return (size_t)cap * (8 * W + 4) + 4096 * 4 + 32 * 4 + 16;
}

size_t seg_sort_lds(int W) {
    int cap = W == 1 ? 11840 : (W == 2 ? 6144 : (W == 3 ? 4480 : 3584));
    return (size_t)cap * (8 * W + 2) + (size_t)2 * kSegWaves * 256 * 4 + 512 * 4 + 2 * 4 * kSegWaves * 8 + 64;
}

// Output of a sorted record: SoA (okeys/ocnts) or, when `packed` is given,
// straight into SortedKMerFile layout (W LE u64 words + LE u32 count).
template <int W>
__device__ __forceinline__ void seg_put(u64* __restrict__ okeys, u32* __restrict__ ocnts, u64 ostride,
                                        u32* __restrict__ packed, u64 pos, const u64 (&k)[W], u32 cnt) {
    if (packed) {
        u32* o = packed + pos * (2 * W + 1);
#pragma unroll
        for (int j = 0; j < W; j++) {
            o[2 * j] = (u32)k[j];
            o[2 * j + 1] = (u32)(k[j] >> 32);
        }
        o[2 * W] = cnt;
    } else {
#pragma unroll
        for (int j = 0; j < W; j++) okeys[(u64)j * ostride + pos] = k[j];
        ocnts[pos] = cnt;
    }
}

constexpr u64 kM48 = 0xffffffffffffull;

__device__ __forceinline__ u32 seg_digit(u64 w0, u64 base, int sh) {
    return (u32)(((w0 & kM48) - base) >> sh) & 4095u;
}

// MSD segment sort: the bits just below the bucket prefix and the pass's
// sub-range bits (known from the descriptor) give a 12-bit digit; a counting
// pass and a scatter pass stream the segment from global memory (L2-resident
// after the first), bins are insertion-sorted by their owner thread. Keys are
// distinct, so the unstable LDS-atomic placement is fine. A segment whose
// largest bin exceeds kMaxBin (skewed keys) is left to seg_sort_lsd_k.
template <int W>
__global__ __launch_bounds__(kSegBlock) void seg_sort_k(const u64* __restrict__ rkeys, const u32* __restrict__ rcnts,
                                                        u64 rstride, const u32* __restrict__ order,
                                                        const u64* __restrict__ dstart, const u32* __restrict__ dlen,
                                                        const u64* __restrict__ out_off, u64 ndesc,
                                                        u64* __restrict__ okeys, u32* __restrict__ ocnts,
                                                        u64 ostride, u32* __restrict__ packed,
                                                        u64* __restrict__ stats, u32* __restrict__ fb,
                                                        u64* __restrict__ fb_n, int skip,
                                                        const u64* __restrict__ dkey) {
    constexpr int CAP = SegCfg<W>::CAP;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64* skey = (u64*)smem;                      // W x CAP
    u32* scnt = (u32*)(skey + (size_t)W * CAP);  // CAP counts, moved with their keys
    u32* bcnt = scnt + CAP;                      // 4096 bins
    u32* misc = bcnt + 4096;                                           // [0] skew flag, [1..16] wave sums
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    // the segment's first PI items per thread (6144 / W records: every segment
    // of a balanced input) are loaded into registers one segment ahead, so
    // the counting and scatter passes do not wait on memory; longer
    // segments read the rest in place
    constexpr int ITEMS = SegCfg<W>::ITEMS;
    constexpr int PI = ITEMS < 6 / W ? ITEMS : 6 / W;
    u64 nk[PI][W];
    u32 nc[PI];
    auto load_seg = [&](u64 d) {
        u64 s0 = 0;
        u32 l0 = 0;
        if (d < ndesc) {
            const u32 od = order[d];
            s0 = dstart[od];
            l0 = dlen[od] & 0xffffffu;
            if (l0 > (u32)CAP) l0 = 0;
        }
        // unconditional loads (clamped into the segment; none past it is used)
#pragma unroll
        for (int i = 0; i < PI; i++) {
            const u32 p = l0 ? min((u32)tid + (u32)i * kSegBlock, l0 - 1) : 0u;
#pragma unroll
            for (int j = 0; j < W; j++) nk[i][j] = rkeys[(u64)j * rstride + s0 + p];
            nc[i] = rcnts[s0 + p];
        }
    };
    load_seg(blockIdx.x);
    for (u64 di = blockIdx.x; di < ndesc; di += gridDim.x) {
        const u32 o = order[di];
        const u64 st = dstart[o];
        const u32 lw = dlen[o];
        const u32 len = lw & 0xffffffu;
        const u64 obase = out_off[di];
        // digit = ((word0 & M48) - base) >> sh: the segment's key range over
        // the 4096 bins (base: the sorted descriptor key's bits below 48)
        const int sh = (int)(lw >> 24) & 63;
        const u64 dbase = dkey ? (dkey[di] & kM48) : 0ull;
        u64 ck[PI][W];
        u32 cc[PI];
#pragma unroll
        for (int i = 0; i < PI; i++) {
#pragma unroll
            for (int j = 0; j < W; j++) ck[i][j] = nk[i][j];
            cc[i] = nc[i];
        }
        load_seg(di + gridDim.x);
        if (lw >> 31) {
            // already sorted (sort_runs_k): copied to its place
#pragma unroll
            for (int i = 0; i < PI; i++) {
                const u32 p = (u32)tid + (u32)i * kSegBlock;
                if (p < len && !(skip & 1)) seg_put<W>(okeys, ocnts, ostride, packed, obase + p, ck[i], cc[i]);
            }
            for (u32 p = tid + PI * kSegBlock; p < ((skip & 1) ? 0u : len); p += kSegBlock) {
                u64 kk[W];
#pragma unroll
                for (int j = 0; j < W; j++) kk[j] = rkeys[(u64)j * rstride + st + p];
                seg_put<W>(okeys, ocnts, ostride, packed, obase + p, kk, rcnts[st + p]);
            }
            continue;
        }
        for (int i = tid; i < 4096; i += kSegBlock) bcnt[i] = 0;
        if (tid == 0) misc[0] = 0;
        __syncthreads();
        if (len > (u32)CAP) {
            if (tid == 0) atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)ERR_SEG_TOO_LONG);
            __syncthreads();
            continue;
        }
#pragma unroll
        for (int i = 0; i < PI; i++)
            if ((u32)tid + (u32)i * kSegBlock < len) atomicAdd(&bcnt[seg_digit(ck[i][0], dbase, sh)], 1u);
        for (u32 p = tid + PI * kSegBlock; p < len; p += kSegBlock)
            atomicAdd(&bcnt[seg_digit(rkeys[st + p], dbase, sh)], 1u);
        __syncthreads();
        // bin starts: 4 bins per thread, block-wide exclusive scan; skew check
        const u32 c0 = bcnt[4 * tid], c1 = bcnt[4 * tid + 1], c2 = bcnt[4 * tid + 2], c3 = bcnt[4 * tid + 3];
        const u32 sum = c0 + c1 + c2 + c3;
        u32 inc = sum;
#pragma unroll
        for (int o2 = 1; o2 < 64; o2 <<= 1) {
            const u32 y = __shfl_up(inc, o2);
            if (lane >= o2) inc += y;
        }
        if (lane == 63) misc[1 + wave] = inc;
        if (max(max(c0, c1), max(c2, c3)) > kMaxBin) atomicOr(&misc[0], 1u);
        __syncthreads();
        if (uni32(misc[0])) {
            if (tid == 0) {
                const u64 f = atomicAdd((unsigned long long*)fb_n, 1ull);
                fb[f] = (u32)di;
            }
            __syncthreads();
            continue;
        }
        u32 wpre = 0;
        for (int w = 0; w < wave; w++) wpre += misc[1 + w];
        const u32 bs = wpre + inc - sum;  // start of this thread's first bin
        bcnt[4 * tid] = bs;
        bcnt[4 * tid + 1] = bs + c0;
        bcnt[4 * tid + 2] = bs + c0 + c1;
        bcnt[4 * tid + 3] = bs + c0 + c1 + c2;
        __syncthreads();
        // scatter into bins (bcnt becomes each bin's end)
#pragma unroll
        for (int i = 0; i < PI; i++) {
            if ((u32)tid + (u32)i * kSegBlock >= len) continue;
            const u32 q = atomicAdd(&bcnt[seg_digit(ck[i][0], dbase, sh)], 1u);
#pragma unroll
            for (int j = 0; j < W; j++) skey[(size_t)j * CAP + q] = ck[i][j];
            scnt[q] = cc[i];
        }
        for (u32 p = tid + PI * kSegBlock; p < len; p += kSegBlock) {
            u64 k[W];
#pragma unroll
            for (int j = 0; j < W; j++) k[j] = rkeys[(u64)j * rstride + st + p];
            const u32 q = atomicAdd(&bcnt[seg_digit(k[0], dbase, sh)], 1u);
#pragma unroll
            for (int j = 0; j < W; j++) skey[(size_t)j * CAP + q] = k[j];
            scnt[q] = rcnts[st + p];
        }
        __syncthreads();
        if constexpr (W == 1) {
            // one-word keys: every record's rank inside its bin (bin d spans
            // [end of bin d - 1, end of bin d) after the scatter; equal keys,
            // which batches that are summed later can hold, by LDS position)
            // is its place: written straight there
            for (u32 p = tid; p < ((skip & 1) ? 0u : len); p += kSegBlock) {
                const u64 kp = skey[p];
                const u32 d = seg_digit(kp, dbase, sh);
                const u32 b0 = d ? bcnt[d - 1] : 0u, b1 = bcnt[d];
                u32 r = 0;
                for (u32 q = b0; q < ((skip & 2) ? b0 : b1); q++) {
                    const u64 kq = skey[q];
                    r += (kq < kp || (kq == kp && q < p)) ? 1u : 0u;
                }
                const u64 kk[1] = {kp};
                seg_put<1>(okeys, ocnts, ostride, packed, obase + b0 + r, kk, scnt[p]);
            }
            __syncthreads();
            continue;
        }
        // insertion sort of this thread's 4 bins [bs, bs + sum)
        const u32 ends[4] = {bs + c0, bs + c0 + c1, bs + c0 + c1 + c2, bs + sum};
        u32 s0 = bs;
        for (int qb = 0; qb < ((skip & 2) ? 0 : 4); qb++) {
            const u32 e0 = ends[qb];
            for (u32 x = s0 + 1; x < e0; x++) {
                u64 kx[W];
#pragma unroll
                for (int jj = 0; jj < W; jj++) kx[jj] = skey[(size_t)jj * CAP + x];
                const u32 ix = scnt[x];
                u32 y = x;
                while (y > s0) {
                    bool less = false, eq = true;
#pragma unroll
                    for (int jj = 0; jj < W; jj++) {
                        const u64 ky = skey[(size_t)jj * CAP + y - 1];
                        if (eq && kx[jj] != ky) {
                            less = kx[jj] < ky;
                            eq = false;
                        }
                    }
                    if (!less) break;
#pragma unroll
                    for (int jj = 0; jj < W; jj++) skey[(size_t)jj * CAP + y] = skey[(size_t)jj * CAP + y - 1];
                    scnt[y] = scnt[y - 1];
                    y--;
                }
#pragma unroll
                for (int jj = 0; jj < W; jj++) skey[(size_t)jj * CAP + y] = kx[jj];
                scnt[y] = ix;
            }
            s0 = e0;
        }
        __syncthreads();
        for (u32 p = tid; p < ((skip & 1) ? 0u : len); p += kSegBlock) {
            u64 kk[W];
#pragma unroll
            for (int jj = 0; jj < W; jj++) kk[jj] = skey[(size_t)jj * CAP + p];
            seg_put<W>(okeys, ocnts, ostride, packed, obase + p, kk, scnt[p]);
        }
        __syncthreads();
    }
}

// LSD fallback for segments with a bin larger than kMaxBin (skewed keys):
// radix passes over the varying bytes with stable wave-private ranking.
template <int W>
__global__ __launch_bounds__(kSegBlock) void seg_sort_lsd_k(const u64* __restrict__ rkeys, const u32* __restrict__ rcnts,
                                                        u64 rstride, const u32* __restrict__ order,
                                                        const u64* __restrict__ dstart, const u32* __restrict__ dlen,
                                                        const u64* __restrict__ out_off, u64 ndesc,
                                                        u64* __restrict__ okeys, u32* __restrict__ ocnts,
                                                        u64 ostride, u32* __restrict__ packed,
                                                        u64* __restrict__ stats,
                                                        const u32* __restrict__ fb, const u64* __restrict__ fb_n) {
    constexpr int CAP = SegCfg<W>::CAP;
    constexpr int ITEMS = SegCfg<W>::ITEMS;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64* skey = (u64*)smem;                                 // W x CAP
    unsigned short* sidx = (unsigned short*)(skey + (size_t)W * CAP);  // CAP
    u32* wcnt = (u32*)(sidx + CAP);                         // kSegWaves x 256
    u32* woff = wcnt + kSegWaves * 256;                     // kSegWaves x 256
    u32* dtot = woff + kSegWaves * 256;                     // 256 digit totals
    u32* dst0 = dtot + 256;                                 // 256 digit starts
    u64* red = (u64*)(dst0 + 256);                          // 2W x kSegWaves reduction scratch
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const u64 lt = lanemask_lt();
    for (int i = tid; i < kSegWaves * 256; i += kSegBlock) wcnt[i] = 0;
    __syncthreads();
    const u64 nfb = *fb_n;
    for (u64 fi = blockIdx.x; fi < nfb; fi += gridDim.x) {
        const u64 di = fb[fi];
        const u32 o = order[di];
        const u64 st = dstart[o];
        const u32 len = dlen[o] & 0xffffffu;
        const u64 obase = out_off[di];
        // blocked-by-wave, lane-striped items over R = ceil(len / 1024) rounds:
        // position p = wave*64*R + it*64 + lane, so every wave holds a share
        const int R = (int)((len + kSegBlock - 1) / kSegBlock);
        u64 key[ITEMS][W];
        unsigned short idx[ITEMS];
        u64 orr[W], andd[W];
#pragma unroll
        for (int j = 0; j < W; j++) {
            orr[j] = 0;
            andd[j] = ~0ull;
        }
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const u32 p = (u32)(wave * 64 * R + it * 64 + lane);
            const bool ok = it < R && p < len;
#pragma unroll
            for (int j = 0; j < W; j++) {
                key[it][j] = ok ? rkeys[(u64)j * rstride + st + p] : ~0ull;
                if (ok) {
                    orr[j] |= key[it][j];
                    andd[j] &= key[it][j];
                }
            }
            idx[it] = (unsigned short)p;
        }
        if (len > (u32)CAP) {
            if (tid == 0) atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)ERR_SEG_TOO_LONG);
            continue;
        }
        // bytes that vary inside the segment
#pragma unroll
        for (int j = 0; j < W; j++) {
            for (int o2 = 32; o2 >= 1; o2 >>= 1) {
                orr[j] |= __shfl_xor(orr[j], o2);
                andd[j] &= __shfl_xor(andd[j], o2);
            }
            if (lane == 0) {
                red[j * kSegWaves + wave] = orr[j];
                red[(W + j) * kSegWaves + wave] = andd[j];
            }
        }
        __syncthreads();
        u64 diff[W];
#pragma unroll
        for (int j = 0; j < W; j++) {
            u64 oo = 0, aa = ~0ull;
            for (int w = 0; w < kSegWaves; w++) {
                oo |= red[j * kSegWaves + w];
                aa &= red[(W + j) * kSegWaves + w];
            }
            diff[j] = oo ^ aa;
        }
        __syncthreads();
        for (int j = W - 1; j >= 0; j--) {
            u64 dj = 0;
#pragma unroll
            for (int jj = 0; jj < W; jj++)
                if (jj == j) dj = diff[jj];
            for (int sh = 0; sh < 64; sh += 8) {
                if (((dj >> sh) & 0xffull) == 0) continue;  // block-uniform
                u32 dig[ITEMS], rank[ITEMS];
#pragma unroll
                for (int it = 0; it < ITEMS; it++) {
                    if (it >= R) break;  // block-uniform
                    const u32 p = (u32)(wave * 64 * R + it * 64 + lane);
                    const bool ok = p < len;
                    u64 kw = key[it][0];
#pragma unroll
                    for (int jj = 1; jj < W; jj++)
                        if (jj == j) kw = key[it][jj];
                    const u32 d = (u32)(kw >> sh) & 255u;
                    dig[it] = d;
                    u64 peers = __ballot(ok);
#pragma unroll
                    for (int bb = 0; bb < 8; bb++) {
                        const u64 m = __ballot((d >> bb) & 1u);
                        peers &= ((d >> bb) & 1u) ? m : ~m;
                    }
                    const u32 before = (u32)__popcll(peers & lt);
                    const u32 base = ok ? wcnt[wave * 256 + d] : 0u;
                    if (ok && before == 0) wcnt[wave * 256 + d] = base + (u32)__popcll(peers);
                    rank[it] = base + before;
                }
                __syncthreads();
                if (tid < 256) {
                    u32 run = 0;
                    for (int w = 0; w < kSegWaves; w++) {
                        const u32 cc = wcnt[w * 256 + tid];
                        woff[w * 256 + tid] = run;
                        wcnt[w * 256 + tid] = 0;
                        run += cc;
                    }
                    dtot[tid] = run;
                }
                __syncthreads();
                if (wave == 0) {
                    // exclusive scan of the 256 digit totals: 4 per lane, no barrier
                    const u32 v0 = dtot[4 * lane], v1 = dtot[4 * lane + 1], v2 = dtot[4 * lane + 2],
                              v3 = dtot[4 * lane + 3];
                    const u32 sum = v0 + v1 + v2 + v3;
                    u32 inc = sum;
#pragma unroll
                    for (int o2 = 1; o2 < 64; o2 <<= 1) {
                        const u32 y = __shfl_up(inc, o2);
                        if (lane >= o2) inc += y;
                    }
                    const u32 ex = inc - sum;
                    dst0[4 * lane] = ex;
                    dst0[4 * lane + 1] = ex + v0;
                    dst0[4 * lane + 2] = ex + v0 + v1;
                    dst0[4 * lane + 3] = ex + v0 + v1 + v2;
                }
                __syncthreads();
#pragma unroll
                for (int it = 0; it < ITEMS; it++) {
                    const u32 p = (u32)(wave * 64 * R + it * 64 + lane);
                    if (it < R && p < len) {
                        const u32 q = dst0[dig[it]] + woff[wave * 256 + dig[it]] + rank[it];
#pragma unroll
                        for (int jj = 0; jj < W; jj++) skey[(size_t)jj * CAP + q] = key[it][jj];
                        sidx[q] = idx[it];
                    }
                }
                __syncthreads();
#pragma unroll
                for (int it = 0; it < ITEMS; it++) {
                    const u32 p = (u32)(wave * 64 * R + it * 64 + lane);
                    if (it < R && p < len) {
#pragma unroll
                        for (int jj = 0; jj < W; jj++) key[it][jj] = skey[(size_t)jj * CAP + p];
                        idx[it] = sidx[p];
                    }
                }
                __syncthreads();
            }
        }
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const u32 p = (u32)(wave * 64 * R + it * 64 + lane);
            if (it < R && p < len) {
                seg_put<W>(okeys, ocnts, ostride, packed, obase + p, key[it], rcnts[st + idx[it]]);
            }
        }
    }
}

hipError_t launch_seg_sort(int W, const uint64_t* rkeys, const uint32_t* rcnts, uint64_t rstride, const uint32_t* order,
                           const uint64_t* dstart, const uint32_t* dlen, const uint64_t* out_off, uint64_t ndesc,
                           uint64_t* okeys, uint32_t* ocnts, uint64_t ostride, uint64_t* stats, uint32_t* fb,
                           uint64_t* fb_n, int grid, hipStream_t s, void* packed, const uint64_t* dkey) {
    if (ndesc == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(fb_n, 0, 8, s);
    if (e != hipSuccess) return e;
    const size_t lds_msd = (seg_sort_msd_lds(W) + 15) & ~(size_t)15;
    const size_t lds = (seg_sort_lds(W) + 15) & ~(size_t)15;
    const int skip = experiment_knob("KC_SEG_SKIP");  // 1 output stores, 2 insertion sort
#define KC_SEG(WW)                                                                                                  \
    hipLaunchKernelGGL(seg_sort_k<WW>, dim3(grid), dim3(kSegBlock), lds_msd, s, rkeys, rcnts, rstride, order,       \
                       dstart, dlen, out_off, ndesc, okeys, ocnts, ostride, (u32*)packed, stats, fb, fb_n, skip,  \
                       dkey);                                                                                      \
    hipLaunchKernelGGL(seg_sort_lsd_k<WW>, dim3(grid), dim3(kSegBlock), lds, s, rkeys, rcnts, rstride, order,       \
                       dstart, dlen, out_off, ndesc, okeys, ocnts, ostride, (u32*)packed, stats, (const u32*)fb,   \
                       (const u64*)fb_n)
    switch (W) {
    case 1: KC_SEG(1); break;
    case 2: KC_SEG(2); break;
    case 3: KC_SEG(3); break;
    case 4: KC_SEG(4); break;
    default: return hipErrorInvalidValue;
    }
#undef KC_SEG
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Key-space partition: owner(key) = ((word0 >> 32) * world)
// >> 32 is monotone in the key, so the owners of a sorted record run are
// contiguous ranges; received runs are unpacked, re-sorted and summed.
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void owner_bounds_k(const uint8_t* __restrict__ packed, int rs, u64 n,
                                                         u32 world, u64* __restrict__ bounds) {
    for (u32 o = blockIdx.x * kBlock + threadIdx.x; o <= world; o += gridDim.x * kBlock) {
        u64 lo = 0, hi = n;
        while (lo < hi) {
            u64 mid = (lo + hi) >> 1;
            const u32* w = (const u32*)(packed + mid * (u64)rs);
            u64 top = w[1];  // high half of word 0 (little endian)
            u32 owner = (u32)((top * world) >> 32);
            if (owner < o)
                lo = mid + 1;
            else
                hi = mid;
        }
        bounds[o] = lo;
    }
}

hipError_t launch_owner_bounds(const void* packed, int rs, uint64_t n, uint32_t world, uint64_t* bounds,
                               hipStream_t s) {
    hipLaunchKernelGGL(owner_bounds_k, dim3(1), dim3(kBlock), 0, s, (const uint8_t*)packed, rs, n, world, bounds);
    return hipGetLastError();
}

template <int W>
__global__ __launch_bounds__(kBlock) void unpack_records_k(const u32* __restrict__ in, u64 n, u64* __restrict__ keys,
                                                           u64 stride, u32* __restrict__ cnts) {
    constexpr int RW = 2 * W + 1;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
        const u32* r = in + i * RW;
#pragma unroll
        for (int j = 0; j < W; j++) keys[(u64)j * stride + i] = (u64)r[2 * j] | ((u64)r[2 * j + 1] << 32);
        cnts[i] = r[2 * W];
    }
}

// ---------------------------------------------------------------------------
// Merge path: two sorted SoA record runs A, B -> one sorted run (A first on
// equal keys; equal keys stay adjacent for the segmented reduce). Tiles of
// kMergeTile outputs: merge_split_k finds each tile's split (i from A) by a
// binary search on the cross diagonal; merge_tile_k loads the tile's A and B
// slices into LDS and every thread merges kMergeItems consecutive outputs.
// ---------------------------------------------------------------------------

template <int W>
struct MergeCfg {
    static constexpr int ITEMS = W <= 2 ? 8 : 4;  // outputs per thread
    static constexpr int TILE = kBlock * ITEMS;   // LDS: TILE x (8W + 4) B <= 40 KB
};
int merge_tile(int W) { return kBlock * (W <= 2 ? 8 : 4); }

template <int W>
__device__ __forceinline__ bool key_le(const u64* __restrict__ ka, u64 sa, u64 ia, const u64* __restrict__ kb, u64 sb,
                                       u64 ib) {
#pragma unroll
    for (int j = 0; j < W; j++) {
        const u64 x = ka[(u64)j * sa + ia], y = kb[(u64)j * sb + ib];
        if (x != y) return x < y;
    }
    return true;
}

template <int W>
__device__ __forceinline__ u64 merge_search(const u64* __restrict__ ka, u64 sa, u64 na, const u64* __restrict__ kb,
                                            u64 sb, u64 nb, u64 diag) {
    u64 lo = diag > nb ? diag - nb : 0, hi = diag < na ? diag : na;
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (key_le<W>(ka, sa, mid, kb, sb, diag - 1 - mid))
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

template <int W>
__global__ __launch_bounds__(kBlock) void merge_split_k(const u64* __restrict__ ka, u64 sa, u64 na,
                                                        const u64* __restrict__ kb, u64 sb, u64 nb, u64 ntiles,
                                                        u64* __restrict__ split) {
    constexpr int TILE = MergeCfg<W>::TILE;
    for (u64 t = (u64)blockIdx.x * kBlock + threadIdx.x; t <= ntiles; t += (u64)gridDim.x * kBlock)
        split[t] = merge_search<W>(ka, sa, na, kb, sb, nb, min(t * (u64)TILE, na + nb));
}

template <int W>
__global__ __launch_bounds__(kBlock) void merge_tile_k(const u64* __restrict__ ka, const u32* __restrict__ ca, u64 sa,
                                                       u64 na, const u64* __restrict__ kb, const u32* __restrict__ cb,
                                                       u64 sb, u64 nb, const u64* __restrict__ split, u64 ntiles,
                                                       u64* __restrict__ ko, u32* __restrict__ co, u64 so) {
    constexpr int kMergeTile = MergeCfg<W>::TILE;
    constexpr int kMergeItems = MergeCfg<W>::ITEMS;
    __shared__ u64 sk[W * kMergeTile];
    __shared__ u32 sc[kMergeTile];
    const int tid = threadIdx.x;
    for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const u64 d0 = t * (u64)kMergeTile, d1 = min(d0 + kMergeTile, na + nb);
        const u64 i0 = split[t], i1 = split[t + 1];
        const u64 j0 = d0 - i0, j1 = d1 - i1;
        const u32 la = (u32)(i1 - i0), lb = (u32)(j1 - j0);
        // LDS: A slice at [0, la), B slice at [la, la + lb)
        for (u32 x = tid; x < la + lb; x += kBlock) {
            const bool fa = x < la;
            const u64 src = fa ? i0 + x : j0 + (x - la);
#pragma unroll
            for (int j = 0; j < W; j++) sk[j * kMergeTile + x] = fa ? ka[(u64)j * sa + src] : kb[(u64)j * sb + src];
            sc[x] = fa ? ca[src] : cb[src];
        }
        __syncthreads();
        // this thread's outputs [dl, dl + kMergeItems) of the tile
        const u32 dl = min((u32)tid * kMergeItems, la + lb);
        u32 lo = dl > lb ? dl - lb : 0, hi = dl < la ? dl : la;
        while (lo < hi) {
            const u32 mid = (lo + hi) >> 1;
            if (key_le<W>(sk, kMergeTile, mid, sk, kMergeTile, la + dl - 1 - mid))
                lo = mid + 1;
            else
                hi = mid;
        }
        u32 ia = lo, ib = dl - lo;
        const u32 de = min(dl + kMergeItems, la + lb);
        for (u32 d = dl; d < de; d++) {
            const bool takea = ib >= lb || (ia < la && key_le<W>(sk, kMergeTile, ia, sk, kMergeTile, la + ib));
            const u32 x = takea ? ia : la + ib;
            if (takea)
                ia++;
            else
                ib++;
#pragma unroll
            for (int j = 0; j < W; j++) ko[(u64)j * so + d0 + d] = sk[j * kMergeTile + x];
            co[d0 + d] = sc[x];
        }
        __syncthreads();
    }
}

hipError_t launch_merge(int W, const uint64_t* ka, const uint32_t* ca, uint64_t sa, uint64_t na, const uint64_t* kb,
                        const uint32_t* cb, uint64_t sb, uint64_t nb, uint64_t* ko, uint32_t* co, uint64_t so,
                        uint64_t* split, hipStream_t s) {
    const u64 n = na + nb;
    if (n == 0) return hipSuccess;
    const u64 ntiles = (n + merge_tile(W) - 1) / merge_tile(W);
    const int gs = (int)hmin((ntiles + 1 + kBlock - 1) / kBlock, 4096);
    const int gt = (int)hmin(ntiles, 8192);
#define KC_MG(WW)                                                                                                    \
    hipLaunchKernelGGL(merge_split_k<WW>, dim3(gs), dim3(kBlock), 0, s, ka, sa, na, kb, sb, nb, ntiles, split);     \
    hipLaunchKernelGGL(merge_tile_k<WW>, dim3(gt), dim3(kBlock), 0, s, ka, ca, sa, na, kb, cb, sb, nb,             \
                       (const u64*)split, ntiles, ko, co, so)
    switch (W) {
    case 1: KC_MG(1); break;
    case 2: KC_MG(2); break;
    case 3: KC_MG(3); break;
    case 4: KC_MG(4); break;
    default: return hipErrorInvalidValue;
    }
#undef KC_MG
    return hipGetLastError();
}

uint64_t merge_split_elems(uint64_t n) { return n / 1024 + 2; }

// ---------------------------------------------------------------------------
// Merge path over packed runs (SortedKMerFile records: W LE u64 key words +
// LE u32 count, RW = 2W + 1 u32 per record), without unpacking: two sorted,
// deduplicated runs A, B -> one sorted packed run (A first on equal keys). A
// key present in both runs leaves two adjacent records; *dup is then set and
// the caller sums them. Tiles of TILE outputs: merge_split_packed_k finds each
// tile's split by a binary search on the cross diagonal; merge_tile_packed_k
// stages the tile's A and B slices in LDS (coalesced u32 copies), every
// thread merges ITEMS consecutive outputs into an LDS staging tile, which is
// copied out with coalesced u32 stores.
// ---------------------------------------------------------------------------

template <int W>
struct MergePkCfg {
    static constexpr int RW = 2 * W + 1;
    static constexpr int ITEMS = W <= 2 ? 8 : 4;
    static constexpr int TILE = kBlock * ITEMS;
};

template <int W>
__device__ __forceinline__ bool pk_le(const u32* __restrict__ a, const u32* __restrict__ b) {
#pragma unroll
    for (int j = 0; j < W; j++) {
        const u64 x = (u64)a[2 * j] | ((u64)a[2 * j + 1] << 32);
        const u64 y = (u64)b[2 * j] | ((u64)b[2 * j + 1] << 32);
        if (x != y) return x < y;
    }
    return true;
}

template <int W>
__device__ __forceinline__ bool pk_eq(const u32* __restrict__ a, const u32* __restrict__ b) {
#pragma unroll
    for (int j = 0; j < 2 * W; j++)
        if (a[j] != b[j]) return false;
    return true;
}

template <int W>
__global__ __launch_bounds__(kBlock) void merge_split_packed_k(const u32* __restrict__ A, u64 na,
                                                               const u32* __restrict__ B, u64 nb, u64 ntiles,
                                                               u64* __restrict__ split) {
    constexpr int RW = MergePkCfg<W>::RW;
    constexpr u64 TILE = MergePkCfg<W>::TILE;
    for (u64 t = (u64)blockIdx.x * kBlock + threadIdx.x; t <= ntiles; t += (u64)gridDim.x * kBlock) {
        const u64 diag = min(t * TILE, na + nb);
        u64 lo = diag > nb ? diag - nb : 0, hi = diag < na ? diag : na;
        while (lo < hi) {
            const u64 mid = (lo + hi) >> 1;
            if (pk_le<W>(A + mid * RW, B + (diag - 1 - mid) * RW))
                lo = mid + 1;
            else
                hi = mid;
        }
        split[t] = lo;
    }
}

template <int W>
__global__ __launch_bounds__(kBlock) void merge_tile_packed_k(const u32* __restrict__ A, u64 na,
                                                              const u32* __restrict__ B, u64 nb,
                                                              const u64* __restrict__ split, u64 ntiles,
                                                              u32* __restrict__ out, u32* __restrict__ dup) {
    constexpr int RW = MergePkCfg<W>::RW;
    constexpr int ITEMS = MergePkCfg<W>::ITEMS;
    constexpr int TILE = MergePkCfg<W>::TILE;
    constexpr int NPT = TILE * RW / kBlock;  // u32 of a tile per thread
    static_assert(TILE * RW % kBlock == 0 && TILE * RW * 4 % 16 == 0, "tile layout");
    __shared__ __attribute__((aligned(16))) u32 sin[TILE * RW];   // A slice, then B slice
    __shared__ __attribute__((aligned(16))) u32 sout[TILE * RW];  // merged tile
    const int tid = threadIdx.x;
    bool seen_dup = false;
    // the next tile's A and B slices are loaded into registers while the
    // current tile merges (software pipeline over the block's tiles)
    u32 v[NPT];
    auto fetch = [&](u64 t) {
        if (t >= ntiles) return;
        const u64 d0 = t * (u64)TILE, d1 = min(d0 + TILE, na + nb);
        const u64 i0 = split[t], i1 = split[t + 1];
        const u32 ea = (u32)(i1 - i0) * RW, tot = (u32)(d1 - d0) * RW;
        const u32* pa = A + i0 * RW;
        const u32* pb = B + (d0 - i0) * RW;
#pragma unroll
        for (int u = 0; u < NPT; u++) {
            const u32 x = (u32)u * kBlock + (u32)tid;
            const u32 xc = min(x, tot - 1);  // unconditional loads (no per-element waits)
            v[u] = __builtin_nontemporal_load(xc < ea ? pa + xc : pb + (xc - ea));
        }
    };
    fetch(blockIdx.x);
    for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const u64 d0 = t * (u64)TILE, d1 = min(d0 + TILE, na + nb);
        const u64 i0 = split[t], i1 = split[t + 1];
        const u64 j0 = d0 - i0, j1 = d1 - i1;
        const u32 la = (u32)(i1 - i0), lb = (u32)(j1 - j0), n = la + lb;
#pragma unroll
        for (int u = 0; u < NPT; u++) {
            const u32 x = (u32)u * kBlock + (u32)tid;
            if (x < n * RW) sin[x] = v[u];
        }
        __syncthreads();
        fetch(t + gridDim.x);
        const u32 dl = min((u32)tid * ITEMS, n);
        u32 lo = dl > lb ? dl - lb : 0, hi = dl < la ? dl : la;
        while (lo < hi) {
            const u32 mid = (lo + hi) >> 1;
            if (pk_le<W>(sin + mid * RW, sin + (la + dl - 1 - mid) * RW))
                lo = mid + 1;
            else
                hi = mid;
        }
        u32 ia = lo, ib = dl - lo;
        const u32 de = min(dl + ITEMS, n);
        for (u32 d = dl; d < de; d++) {
            const bool takea = ib >= lb || (ia < la && pk_le<W>(sin + ia * RW, sin + (la + ib) * RW));
            const u32 x = takea ? ia : la + ib;
            if (takea)
                ia++;
            else
                ib++;
#pragma unroll
            for (int j = 0; j < RW; j++) sout[d * RW + j] = sin[x * RW + j];
        }
        __syncthreads();
        // a key of both runs: two equal neighbours in the output (at the tile
        // start, the neighbour is the larger of A[i0 - 1], B[j0 - 1])
        for (u32 d = tid; d < n; d += kBlock) {
            if (d > 0) {
                seen_dup |= pk_eq<W>(sout + d * RW, sout + (d - 1) * RW);
            } else {
                if (i0 > 0) {
                    u32 p[RW];
#pragma unroll
                    for (int j = 0; j < RW; j++) p[j] = A[(i0 - 1) * RW + j];
                    seen_dup |= pk_eq<W>(sout, p);
                }
                if (j0 > 0) {
                    u32 p[RW];
#pragma unroll
                    for (int j = 0; j < RW; j++) p[j] = B[(j0 - 1) * RW + j];
                    seen_dup |= pk_eq<W>(sout, p);
                }
            }
        }
        u32* o = out + d0 * RW;
        const u32 tot = n * RW;
        if (((uintptr_t)o & 15u) == 0) {  // 16-byte stores (tiles start 16-byte aligned in an aligned run)
            const u32 nv = tot / 4;
            for (u32 x = tid; x < nv; x += kBlock) ((uint4*)o)[x] = ((const uint4*)sout)[x];
            for (u32 x = nv * 4 + tid; x < tot; x += kBlock) o[x] = sout[x];
        } else {
            for (u32 x = tid; x < tot; x += kBlock) o[x] = sout[x];
        }
        __syncthreads();
    }
    if (__ballot(seen_dup) && lane_id() == 0) atomicOr(dup, 1u);
}

hipError_t launch_merge_packed(int W, const void* a, uint64_t na, const void* b, uint64_t nb, void* out,
                               uint64_t* split, uint32_t* dup, hipStream_t s) {
    const u64 n = na + nb;
    if (n == 0) return hipSuccess;
    const u64 tile = (u64)kBlock * (W <= 2 ? 8 : 4);
    const u64 ntiles = (n + tile - 1) / tile;
    const int gs = (int)hmin((ntiles + 1 + kBlock - 1) / kBlock, 4096);
    const int gt = (int)hmin(ntiles, 8192);
#define KC_MGP(WW)                                                                                                \
    hipLaunchKernelGGL(merge_split_packed_k<WW>, dim3(gs), dim3(kBlock), 0, s, (const u32*)a, na, (const u32*)b, \
                       nb, ntiles, split);                                                                        \
    hipLaunchKernelGGL(merge_tile_packed_k<WW>, dim3(gt), dim3(kBlock), 0, s, (const u32*)a, na, (const u32*)b,  \
                       nb, (const u64*)split, ntiles, (u32*)out, dup)
    switch (W) {
    case 1: KC_MGP(1); break;
    case 2: KC_MGP(2); break;
    case 3: KC_MGP(3); break;
    case 4: KC_MGP(4); break;
    default: return hipErrorInvalidValue;
    }
#undef KC_MGP
    return hipGetLastError();
}

uint64_t merge_packed_split_elems(int W, uint64_t n) {
    return n / ((uint64_t)kBlock * (W <= 2 ? 8 : 4)) + 2;
}

hipError_t launch_unpack(int W, const void* packed, uint64_t n, uint64_t* keys, uint64_t stride, uint32_t* cnts,
                         hipStream_t s) {
    if (n == 0) return hipSuccess;
    int g = grid_for(n);
    switch (W) {
    case 1: hipLaunchKernelGGL(unpack_records_k<1>, dim3(g), dim3(kBlock), 0, s, (const u32*)packed, n, keys, stride, cnts); break;
    case 2: hipLaunchKernelGGL(unpack_records_k<2>, dim3(g), dim3(kBlock), 0, s, (const u32*)packed, n, keys, stride, cnts); break;
    case 3: hipLaunchKernelGGL(unpack_records_k<3>, dim3(g), dim3(kBlock), 0, s, (const u32*)packed, n, keys, stride, cnts); break;
    case 4: hipLaunchKernelGGL(unpack_records_k<4>, dim3(g), dim3(kBlock), 0, s, (const u32*)packed, n, keys, stride, cnts); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K1: FASTQ block index. The block is viewed through 16-byte-aligned 64 KiB
// chunks of the address space; fq_count counts '\n' per chunk, a device scan
// turns counts into each chunk's first line index, and fq_emit re-reads the
// chunk and, in address order, gives every newline its line index j:
//   j % 4 == 0 (header ends)   -> seq_off[j/4] = q + 1
//   j % 4 == 1 (sequence ends) -> seq_end[j/4] = q, next byte must be '+'
//   j % 4 == 3 (quality ends)  -> next byte must be '@' (or end of block)
// For well-formed 4-line records this selects exactly the lines readData
// copies (the line before each '+' line, FASTQFileReader.cpp:57-63).
// ---------------------------------------------------------------------------

constexpr u64 kFqChunk = 16384;  // one wave: 64 lanes x 16 B x 16 iterations
constexpr int kFqWaves = kBlock / 64;

uint64_t fq_chunks(const void* base, uint64_t n) {
    u64 lead = (u64)((uintptr_t)base & 15);
    return (lead + n + kFqChunk - 1) / kFqChunk;
}

// Newline bytes of a 16-byte load as a 16-bit mask (bit b = byte b), limited
// to the bytes whose offset rel0 + b lies in [0, n).
__device__ __forceinline__ u32 nl_mask16(const uint4 v, long long rel0, u64 n) {
    u32 m = 0;
    const u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; q++) {
        u32 t = w[q] ^ 0x0a0a0a0au;
        u32 nz = ((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t;  // 0x80 set in non-zero bytes
        u32 z = ~nz & 0x80808080u;                      // 0x80 in '\n' bytes
#pragma unroll
        for (int b = 0; b < 4; b++)
            if (z & (0x80u << (8 * b))) m |= 1u << (4 * q + b);
    }
    if (rel0 < 0) m &= 0xffffu << (u32)(-rel0 > 16 ? 16 : -rel0);
    long long over = rel0 + 16 - (long long)n;
    if (over > 0) m &= (over >= 16) ? 0u : (0xffffu >> (u32)over);
    return m & 0xffffu;
}

// 16 bytes of the block (global address space spelled out: no FLAT load)
__device__ __forceinline__ uint4 fq_load16(uintptr_t addr) {
    const v4u w4 = *(const __attribute__((address_space(1))) v4u*)addr;
    return make_uint4(w4.x, w4.y, w4.z, w4.w);
}

// Every wave counts the newlines of its own chunks (no workgroup barrier).
__global__ __launch_bounds__(kBlock) void fq_count_k(const uint8_t* __restrict__ base, u64 n, u64 nchunks,
                                                     u64* __restrict__ counts) {
    const uintptr_t A = (uintptr_t)base & ~(uintptr_t)15;
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (u64 c = (u64)blockIdx.x * kFqWaves + wave; c < nchunks; c += (u64)gridDim.x * kFqWaves) {
        u32 cnt = 0;
#pragma unroll 4
        for (int it = 0; it < 16; it++) {
            const uintptr_t addr = A + c * kFqChunk + (u64)it * 1024 + (u64)lane * 16;
            const long long rel0 = (long long)(addr - (uintptr_t)base);
            if (rel0 + 16 <= 0 || rel0 >= (long long)n) continue;
            cnt += __popc(nl_mask16(fq_load16(addr), rel0, n));
        }
        for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
        if (lane == 0) counts[c] = cnt;
    }
}

// The byte after byte b of a 16-byte load (at block offset q): from the load
// itself, from the next lane's load (nxw: its first word) for the last byte,
// from memory only at the wave's last lane (the caller checks q + 1 < n).
__device__ __forceinline__ u32 fq_next_byte(const uint4 v, u32 nxw, int b, const uint8_t* __restrict__ base, u64 q) {
    if (b == 15) return lane_id() < 63 ? (nxw & 255u) : (u32)base[q + 1];
    const int i = b + 1;
    const u32 w = (i & 8) ? ((i & 4) ? v.w : v.z) : ((i & 4) ? v.y : v.x);
    return (w >> (8 * (i & 3))) & 255u;
}

// Every wave numbers the newlines of its own chunks from the chunk's line
// base (wave scans only, no workgroup barrier; the next 1 KiB slice is
// loaded while this one is emitted).
__global__ __launch_bounds__(kBlock) void fq_emit_k(const uint8_t* __restrict__ base, u64 n, u64 nchunks,
                                                    const u64* __restrict__ line_base, u64* __restrict__ seq_off,
                                                    u64* __restrict__ seq_end, u64 max_rec, u64* stats) {
    const uintptr_t A = (uintptr_t)base & ~(uintptr_t)15;
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u64 err = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (n == 0 || base[0] != '@') err |= ERR_FQ_NOT_AT;
        if (n > 0 && base[n - 1] != '\n') err |= ERR_FQ_NO_FINAL_NL;
    }
    auto load = [&](u64 c, int it, long long* rel) {
        const uintptr_t addr = A + c * kFqChunk + (u64)it * 1024 + (u64)lane * 16;
        *rel = (long long)(addr - (uintptr_t)base);
        uint4 v = make_uint4(0, 0, 0, 0);
        if (!(*rel + 16 <= 0 || *rel >= (long long)n)) v = fq_load16(addr);
        return v;
    };
    for (u64 c = (u64)blockIdx.x * kFqWaves + wave; c < nchunks; c += (u64)gridDim.x * kFqWaves) {
        u64 run = line_base[c];
        long long reln;
        uint4 vn = load(c, 0, &reln);
        for (int it = 0; it < 16; it++) {
            const uint4 v = vn;
            const long long rel0 = reln;
            if (it < 15) vn = load(c, it + 1, &reln);
            u32 m = (rel0 + 16 <= 0 || rel0 >= (long long)n) ? 0u : nl_mask16(v, rel0, n);
            const u32 nxw = (u32)__shfl_down((int)v.x, 1);
            const u32 cnt = (u32)__popc(m);
            u32 inc = cnt;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const u32 y = __shfl_up(inc, o);
                if (lane >= o) inc += y;
            }
            u64 j = run + (inc - cnt);
            run += (u32)__shfl((int)inc, 63);
            while (m) {
                const int b = __ffs(m) - 1;
                m &= m - 1;
                const u64 q = (u64)(rel0 + b);
                const u64 rec = j >> 2;
                switch (j & 3) {
                case 0:
                    if (rec < max_rec) seq_off[rec] = q + 1;
                    else err |= ERR_FQ_TOO_MANY;
                    break;
                case 1:
                    if (rec < max_rec) seq_end[rec] = q;
                    else err |= ERR_FQ_TOO_MANY;
                    if (q + 1 >= n || fq_next_byte(v, nxw, b, base, q) != '+') err |= ERR_FQ_NO_PLUS;
                    break;
                case 3:
                    if (q + 1 < n && fq_next_byte(v, nxw, b, base, q) != '@') err |= ERR_FQ_NOT_AT;
                    break;
                default: break;
                }
                j++;
            }
        }
    }
    if (err) atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)err);
}

__global__ __launch_bounds__(kBlock) void fq_validate_k(const u64* __restrict__ seq_off,
                                                        const u64* __restrict__ seq_end, u64 n_rec, int L,
                                                        u64* stats, int at_most) {
    bool bad = false;
    for (u64 r = (u64)blockIdx.x * kBlock + threadIdx.x; r < n_rec; r += (u64)gridDim.x * kBlock) {
        const u64 len = seq_end[r] - seq_off[r];
        bad |= at_most ? len > (u64)L : len != (u64)L;
    }
    if (__ballot(bad) && lane_id() == 0)
        atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)ERR_FQ_SEQ_LEN);
}

// K1 emit + E fused (engines that read codes, when the block is one batch):
// fq_emit_k's newline walk and encode_reads_k's encoding with one read of the
// text. Every wave takes its chunk in two halves of 8 KiB. A half and the next
// KiB are staged in the wave's LDS. The half is walked in two rounds of 64
// bytes per lane (one 64-bit newline mask per lane; the lanes' newline counts
// are scanned by ballots of their bits); every newline gets its line index
// from the chunk's line base, the '+' / '@' checks read the staged bytes, and
// the records whose header ends in the half are listed (sequence start per
// record). Then the wave encodes those reads, one (read, 16-base group) per
// lane, from LDS (groups past the staged bytes from global memory) into codes /
// inval at the read's index. The sequence-length check of fq_validate_k is
// done inline: no newline inside [s, s + L) and a newline at s + L, which is
// exactly seq_end - seq_off == L. Nothing is written to seq_off / seq_end.
#ifndef KC_FQ_HALF
#define KC_FQ_HALF 8192  // bytes walked per step (a multiple of 4096 dividing kFqChunk)
#endif
#ifndef KC_FQ_XB
#define KC_FQ_XB 16  // bytes per lane staged past the half (8 or 16)
#endif
#ifndef KC_FQ_BLOCK
#define KC_FQ_BLOCK 256  // fq_encode_k workgroup (small groups: as many resident per CU as registers allow)
#endif
#ifndef KC_FQ_WPE
#define KC_FQ_WPE 1  // fq_encode_k: minimum waves per SIMD asked of the register allocator (1 = no limit)
#endif
constexpr int kFqHalf = KC_FQ_HALF;
constexpr int kFqRounds = kFqHalf / 4096;        // 64 lanes x 64 B per round
constexpr int kFqParts = (int)(kFqChunk / kFqHalf);  // halves per fq_count chunk
constexpr int kFqStage = kFqHalf + 64 * KC_FQ_XB;
constexpr int kFqEncBlock = KC_FQ_BLOCK;
constexpr int kFqEncWaves = kFqEncBlock / 64;
static_assert(kFqRounds >= 1 && kFqHalf % 4096 == 0 && kFqChunk % kFqHalf == 0, "fq half size");
static_assert(KC_FQ_XB == 8 || KC_FQ_XB == 16, "fq extra staging");

int fq_encode_list_cap(int L) { return kFqHalf / (L + 6) + 2; }  // records with an L-base sequence are >= L + 6 bytes

static size_t fq_encode_wave_lds(int L) {
    return (size_t)kFqStage + (((size_t)fq_encode_list_cap(L) * 2 + 15) & ~(size_t)15);
}

// bit b set when byte b of w is '\n'
__device__ __forceinline__ u32 nl_nib(u32 w) {
    const u32 t = w ^ 0x0a0a0a0au;
    const u32 z = ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
    return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | (z >> 28);
}

// '\n' bytes of 16 bytes (4 dwords, first byte lowest) as a 16-bit mask, bit
// i = byte i: the per-byte flags (0x80 per byte) of each dword are weighted
// by v_dot4_u32_u8 (bytes 1 2 4 8 for dwords 0 and 2, 16 32 64 128 for 1 and
// 3, two dwords accumulated per half), so each half is its 8-bit mask times 128
__device__ __forceinline__ u32 nl_mask16w(u32 w0, u32 w1, u32 w2, u32 w3) {
    auto z = [](u32 w) {
        const u32 t = w ^ 0x0a0a0a0au;
        return ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
    };
    const u32 lo = __builtin_amdgcn_udot4(z(w1), 0x80402010u, __builtin_amdgcn_udot4(z(w0), 0x08040201u, 0u, false), false);
    const u32 hi = __builtin_amdgcn_udot4(z(w3), 0x80402010u, __builtin_amdgcn_udot4(z(w2), 0x08040201u, 0u, false), false);
    return (lo >> 7) | (hi << 1);
}

// newline bytes among the first nv bytes of a dword (any)
__device__ __forceinline__ bool has_nl(u32 x, int nv) {
    if (nv <= 0) return false;
    const u32 t = x ^ 0x0a0a0a0au;
    const u32 z = ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
    const u32 vm = nv >= 4 ? 0x80808080u : (0x80808080u >> (8 * (4 - nv)));
    return (z & vm) != 0u;
}

// bytes_to_codes by SWAR: 4 bytes -> 4 2-bit codes in the low byte (first
// byte highest; ((c >> 1) ^ (c >> 2)) & 3 is A0 C1 G2 T3) and the 4-bit
// not-ACGT mask (a byte is ACGT iff it equals the ACGT byte of its code,
// looked up by v_perm); non-ACGT bytes code 3, bytes >= nv code 0 and valid
__device__ __forceinline__ u32 swar_codes(u32 x, int nv, u32* bad4) {
    const u32 vm = nv >= 4 ? ~0u : (nv <= 0 ? 0u : (~0u >> (8 * (4 - nv))));
    u32 t = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
    const u32 y = __builtin_amdgcn_perm(0u, 0x54474341u, t) ^ x;
    const u32 bad = (((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y) & 0x80808080u & vm;
    t = (t & vm) | (bad >> 7) | (bad >> 6);
    *bad4 = ((bad >> 4) & 8u) | ((bad >> 13) & 4u) | ((bad >> 22) & 2u) | (bad >> 31);
    return ((t << 6) | (t >> 4) | (t >> 14) | (t >> 24)) & 255u;
}

// 16 bytes (x0 first, lowest byte first; nb of them valid) -> the group's code
// word (base 0 in bits 31-30) and not-ACGT mask (base 0 in bit 15), as
// swar_codes per dword; each dword's four 2-bit codes and four bad-byte flags
// are packed by one v_dot4_u32_u8 each (bytes times 64 16 4 1 and 8 4 2 1:
// the first byte lands highest)
__device__ __forceinline__ u32 swar_group(u32 x0, u32 x1, u32 x2, u32 x3, int nb, u32* bad16) {
    const u32 xs[4] = {x0, x1, x2, x3};
    u32 code = 0, bm = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int nv = nb - 4 * k;
        const u32 vm = nv >= 4 ? ~0u : (nv <= 0 ? 0u : (~0u >> (8 * (4 - nv))));
        u32 t = ((xs[k] >> 1) ^ (xs[k] >> 2)) & 0x03030303u;
        const u32 y = __builtin_amdgcn_perm(0u, 0x54474341u, t) ^ xs[k];
        const u32 bad = (((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y) & 0x80808080u & vm;
        const u32 b1 = bad >> 7;  // 1 in each bad byte
        t = (t & vm) | b1 | (bad >> 6);  // bad bytes code 3, bytes past nb code 0
        code = __builtin_amdgcn_udot4(t, 0x01041040u, code << 8, false);
        bm = __builtin_amdgcn_udot4(b1, 0x01020408u, bm << 4, false);
    }
    *bad16 = bm;
    return code;
}

// VAR (KC_FLAG_VARLEN): sequences of 0..L bases. After the newline walk one
// lane per listed record finds its sequence's newline (staged dwords, global
// past the staging) and keeps its length; the encode then reads only the
// read's own bytes and marks the rest of the L-base slot not-ACGT (as
// encode_reads_var_k). The list holds lcap records per half (records of >= 32
// bytes); a denser half sets ERR_FQ_LIST.
// SP (one-pass index, fixed L): no line_base. Each chunk guesses its line
// phase (the line index of its first byte mod 4) from the first newlines of
// its text: the line after newline i is taken for a header when a line of L
// bases, a '+' line and a line of L bytes follow (a quality line starting with
// '@' is followed by a header and a sequence line, which does not start with
// '+'). The chunk's records go to its own rows [c cap, c cap + cap) (cap =
// max_rec), the rows past them are empty (rlen 0, codes 0, every base
// not-ACGT), and sp_cnt[c] / sp_phase[c] = its newlines / phase | 4 (not
// found). fq_spec_verify_k checks the phases against the scanned counts; any
// miss or error sends the block to the two-kernel index. rlen[row] = L for the
// records; stats[ST_VHOLE] is set when a read holds a not-ACGT base.
template <bool VAR, bool SP = false>
__global__ __launch_bounds__(kFqEncBlock) __attribute__((amdgpu_waves_per_eu(KC_FQ_WPE))) void fq_encode_k(const uint8_t* __restrict__ base, u64 n, u64 nchunks,
                                                      const u64* __restrict__ line_base, u64 max_rec_in, int L, int G,
                                                      int lcap, u32* __restrict__ codes,
                                                      unsigned short* __restrict__ inval, u64* stats,
                                                      unsigned short* __restrict__ rlen, int k,
                                                      u64* __restrict__ sp_cnt,
                                                      unsigned char* __restrict__ sp_phase) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uintptr_t A = (uintptr_t)base & ~(uintptr_t)15;
    const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u64 lt = lanemask_lt();
    const size_t wbytes = (size_t)kFqStage + (((size_t)lcap * (VAR ? 4 : 2) + 15) & ~(size_t)15);
    unsigned char* txt = smem + (size_t)wave * wbytes;
    unsigned short* lst = (unsigned short*)(txt + kFqStage);
    unsigned short* lenl = lst + lcap;  // VAR: the listed records' sequence lengths
    bool vhole = false;
    u64 vwin = 0;
    const FastDivU divg((u32)G);
    const FastDivU divg1((u32)(G > 1 ? G - 1 : 1));  // fixed L: the full groups of a read
    u64 err = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (n == 0 || base[0] != '@') err |= ERR_FQ_NOT_AT;
        if (n > 0 && base[n - 1] != '\n') err |= ERR_FQ_NO_FINAL_NL;
    }
    auto sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    };
    // the wave's halves in order: (c, 0), (c, 1), (c + stride, 0), ...; the
    // next half's text is loaded into registers while this one is walked and
    // encoded from LDS
    const u64 cstride = (u64)gridDim.x * kFqEncWaves;
    uint4 v[kFqRounds][4], x;
    auto issue = [&](u64 cc, int hh) {
        const uintptr_t hb = A + cc * kFqChunk + (u64)hh * kFqHalf;
        const long long hrel = (long long)(hb - (uintptr_t)base);
#pragma unroll
        for (int rd = 0; rd < kFqRounds; rd++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int o = rd * 4096 + lane * 64 + i * 16;
                const long long rel = hrel + o;
                v[rd][i] = (rel + 16 <= 0 || rel >= (long long)n) ? make_uint4(0, 0, 0, 0) : fq_load16(hb + (u64)o);
            }
        const int o = kFqHalf + lane * KC_FQ_XB;
        const long long rel = hrel + o;
        if constexpr (KC_FQ_XB == 16) {
            x = (rel >= (long long)n) ? make_uint4(0, 0, 0, 0) : fq_load16(hb + (u64)o);
        } else {
            const u64 y0 = rel >= (long long)n ? 0ull : *(const __attribute__((address_space(1))) u64*)(hb + (u64)o);
            x = make_uint4((u32)y0, (u32)(y0 >> 32), 0u, 0u);  // bytes 8..15: no newline
        }
    };
    // a newline mask of 64 staged bytes limited to the block's bytes
    auto trim = [&](u64 m, long long rel0) -> u64 {
        if (rel0 < 0) m = (rel0 <= -64) ? 0ull : (m & (~0ull << (u32)(-rel0)));
        if (rel0 + 64 > (long long)n) m = (rel0 >= (long long)n) ? 0ull : (m & (~0ull >> (u32)(rel0 + 64 - (long long)n)));
        return m;
    };
    u64 c = (u64)blockIdx.x * kFqEncWaves + wave;
    int h = 0;
    u64 run = 0;
    // SP: the chunk's phase, whether it was found, its first record's local
    // index ((phase + 3) >> 2) and the row of local record 0 (row = rowoff + local)
    u32 sp_phi = 0;
    bool sp_fail = false;
    u64 rbase = 0, rowoff = 0;
    u64 max_rec = max_rec_in;
    if constexpr (SP) {
        // rows per chunk for this block: records are at least 2L + 5 + h
        // bytes with h the header line's length; h from the block's first
        // header less a margin (header lengths differ by the read number's
        // digits). A chunk denser than that reports ERR_FQ_TOO_MANY and the
        // block takes the two-kernel index. max_rec_in assumes h = 1.
        u32 h0 = 1;
        bool found = false;
        for (u32 b0 = 0; b0 < 1024u && !found; b0 += 256u) {
            const u64 o = (u64)b0 + 4u * (u32)lane;
            int pos = -1;
#pragma unroll
            for (int b = 3; b >= 0; b--)
                if (o + (u64)b < n && base[o + (u64)b] == (uint8_t)'\n') pos = (int)(o + (u64)b);
            const u64 bm = __ballot(pos >= 0);
            if (bm) {
                h0 = (u32)__builtin_amdgcn_readlane(pos, __ffsll((long long)bm) - 1);
                found = true;
            }
        }
        const u64 hmin = h0 > 17u ? (u64)h0 - 16u : 1u;
        max_rec = min(max_rec_in, 1 + (kFqChunk - 1) / (2 * (u64)L + 5 + hmin));
        if (blockIdx.x == 0 && threadIdx.x == 0) sp_cnt[nchunks + 1] = max_rec;
    }
    if (c < nchunks) issue(c, 0);
    while (c < nchunks) {
        {
            const uintptr_t hb = A + c * kFqChunk + (u64)h * kFqHalf;
            const long long hrel = (long long)(hb - (uintptr_t)base);
            if constexpr (!SP) {
                if (h == 0) run = line_base[c];
            }
            // the next half: (c, 1) unless it starts past the block
            u64 cn = c;
            int hn = 1;
            if (h == kFqParts - 1 || (long long)(hrel + kFqHalf) >= (long long)n) {
                cn = c + cstride;
                hn = 0;
            } else {
                hn = h + 1;
            }
#pragma unroll
            for (int rd = 0; rd < kFqRounds; rd++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    v4u w;
                    w.x = v[rd][i].x;
                    w.y = v[rd][i].y;
                    w.z = v[rd][i].z;
                    w.w = v[rd][i].w;
                    *(v4u*)(txt + rd * 4096 + lane * 64 + i * 16) = w;
                }
            if constexpr (KC_FQ_XB == 16) {
                v4u w;
                w.x = x.x;
                w.y = x.y;
                w.z = x.z;
                w.w = x.w;
                *(v4u*)(txt + kFqHalf + lane * 16) = w;
            } else {
                *(u64*)(txt + kFqHalf + lane * 8) = (u64)x.x | ((u64)x.y << 32);
            }
            u64 mk[kFqRounds];
#pragma unroll
            for (int rd = 0; rd < kFqRounds; rd++) {
                u64 m = 0;
#pragma unroll
                for (int i = 0; i < 4; i++)
                    m |= (u64)nl_mask16w(v[rd][i].x, v[rd][i].y, v[rd][i].z, v[rd][i].w) << (16 * i);
                mk[rd] = m;
            }
            // VAR: newlines of the staged KiB past the half (the sequence end
            // of a record that straddles the half end is its first one); the
            // walk writes each listed record's sequence-end position
            u32 mx = 0;
            if constexpr (VAR) {
                mx = nl_mask16w(x.x, x.y, x.z, x.w);
                for (int i = lane; i < lcap; i += 64) lenl[i] = 0xffffu;
            }
            if (cn < nchunks) issue(cn, hn);
            sync();
            if constexpr (SP) {
                if (h == 0) {
                    // the phase from the first newlines of the chunk's first 4 KiB
                    // (the block's first chunk starts with a header: phase 0)
                    sp_phi = 0;
                    sp_fail = false;
                    if (c != 0) {
                        u64 m0 = trim(mk[0], hrel + lane * 64);
                        const u32 c0 = (u32)__popcll(m0);
                        u32 inc = c0;
#pragma unroll
                        for (int o = 1; o < 64; o <<= 1) {
                            const u32 y = __shfl_up(inc, o);
                            if (lane >= o) inc += y;
                        }
                        u32 kx = inc - c0;
                        const u32 tot0 = (u32)__shfl((int)inc, 63);
                        unsigned short* nl8 = lst;  // scratch: the walk below rewrites the list
                        while (m0 && kx < 8u) {
                            nl8[kx++] = (unsigned short)(lane * 64 + __ffsll((long long)m0) - 1);
                            m0 &= m0 - 1;
                        }
                        sync();
                        sp_fail = true;
                        int nl[8];
#pragma unroll
                        for (int i = 0; i < 8; i++) nl[i] = (u32)i < tot0 ? (int)nl8[i] : 0;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            if (sp_fail && (u32)(i + 4) < tot0 && txt[nl[i] + 1] == (unsigned char)'@' &&
                                nl[i + 2] - nl[i + 1] - 1 == L && txt[nl[i + 2] + 1] == (unsigned char)'+' &&
                                nl[i + 4] - nl[i + 3] - 1 == L) {
                                sp_phi = (u32)(3 - i) & 3u;
                                sp_fail = false;
                            }
                        }
                        sync();
                    }
                    run = sp_phi;
                    rbase = (sp_phi + 3u) >> 2;
                    rowoff = c * max_rec - rbase;
                }
            }
            const u64 rec0 = (run + 3) >> 2;  // first record whose header may end in this half
#pragma unroll
            for (int rd = 0; rd < kFqRounds; rd++) {
                u64 m = mk[rd];
                const long long rel0 = hrel + rd * 4096 + lane * 64;
                m = trim(m, rel0);
                const u32 cnt = (u32)__popcll(m);
                u32 ex = 0, tot = 0;
                if (__ballot(cnt > 7u) == 0ull) {
                    // counts below 8: the prefix from three bit-plane ballots
#pragma unroll
                    for (int bp = 0; bp < 3; bp++) {
                        const u64 bl = __ballot((cnt >> bp) & 1u);
                        ex += (u32)__popcll(bl & lt) << bp;
                        tot += (u32)__popcll(bl) << bp;
                    }
                } else {
                    u32 inc = cnt;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const u32 y = __shfl_up(inc, o);
                        if (lane >= o) inc += y;
                    }
                    ex = inc - cnt;
                    tot = (u32)__shfl((int)inc, 63);
                }
                u64 j = run + ex;
                run += tot;
                while (m) {
                    const int b = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    const int o = rd * 4096 + lane * 64 + b;  // staged position of the newline
                    const u64 q = (u64)(hrel + o);
                    const u32 jc = (u32)j & 3u;
                    if (jc == 0u) {
                        const u64 li = (j >> 2) - rec0;
                        if ((j >> 2) - rbase >= max_rec) err |= ERR_FQ_TOO_MANY;
                        else if (li < (u64)lcap) lst[li] = (unsigned short)(o + 1);
                        else err |= VAR ? ERR_FQ_LIST : ERR_FQ_SEQ_LEN;  // more records than the list holds
                    } else if (jc != 2u) {
                        if (VAR && jc == 1u) {
                            const u64 li = (j >> 2) - rec0;  // wraps for records listed by the previous half
                            if (li < (u64)lcap) lenl[li] = (unsigned short)o;
                        }
                        // after the sequence: '+'; after the quality line: '@' (or the block end)
                        const u32 nx = q + 1 < n ? (u32)txt[o + 1] : 0u;
                        if (jc == 1u ? nx != (u32)'+' : (q + 1 < n && nx != (u32)'@'))
                            err |= jc == 1u ? ERR_FQ_NO_PLUS : ERR_FQ_NOT_AT;
                    }
                    j++;
                }
            }
            sync();
            // records [rec0, rec1) have their header newline in this half
            u64 rec1 = (run + 3) >> 2;
            if (rec1 - rbase > max_rec) rec1 = rbase + max_rec;
            const u32 nrec = rec1 > rec0 ? (u32)min(rec1 - rec0, (u64)lcap) : 0u;
            if constexpr (VAR) {
                // each listed record's sequence length: the walk saw its
                // sequence end, or (at most one record, the one straddling the
                // half end) it is the first newline of the staged KiB past the
                // half, or (reads past that KiB) found by a dword scan
                const u64 bx = __ballot(mx != 0u);
                int ex = -1;
                if (bx) {
                    const int fl = __ffsll((long long)bx) - 1;
                    ex = kFqHalf + KC_FQ_XB * fl + __builtin_ctz((u32)__builtin_amdgcn_readlane((int)mx, fl));
                }
                for (u32 li = (u32)lane; li < nrec; li += 64) {
                    const int s = (int)lst[li];
                    const u32 se = lenl[li];
                    int pos = s & ~3, e = se != 0xffffu ? (int)se : (s <= kFqHalf ? ex : -1);
                    while (e < 0 && pos - s <= L) {
                        u32 w;
                        if (pos + 4 <= kFqStage) {
                            w = *(const u32*)(txt + pos);
                        } else {
                            const long long q = hrel + pos;  // block offset of the dword (4-aligned address)
                            typedef __attribute__((address_space(1))) const u32 g32;
                            w = q < (long long)n ? *(const g32*)(hb + (u64)pos) : 0x0a0a0a0au;
                        }
                        u32 m = nl_nib(w);
                        if (pos < s) m &= 0xfu << (s - pos);
                        if (m) e = pos + __builtin_ctz(m);
                        pos += 4;
                    }
                    const int len = e < 0 ? L + 1 : e - s;
                    if (len > L) err |= ERR_FQ_SEQ_LEN;
                    const int lc = min(len, L);
                    lenl[li] = (unsigned short)lc;
                    if (rlen) rlen[rec0 + li] = (unsigned short)lc;
                    if (lc >= k) vwin += (u64)(lc - k + 1);
                }
                sync();
            }
            // the half's rows start at row rowoff + rec0: item (r, g) is word
            // r G + g = item past that row's first word (no per-item 64-bit math)
            u32* const hcodes = codes + (rowoff + rec0) * (u64)G;
            unsigned short* const hinval = inval + (rowoff + rec0) * (u64)G;
            // group g of listed record r (item r G + g)
            auto encode = [&](u32 r, int g, int nb0, bool lastg) {
                const u32 item = r * (u32)G + (u32)g;
                const int s0 = (int)lst[r] + 16 * g;  // staged offset of the group's first base
                const int lr = VAR ? (int)lenl[r] : L;
                const int nb = VAR ? max(0, min(nb0, lr - 16 * g)) : nb0;  // of them, bases of the read
                const int need = nb + ((lastg && !VAR) ? 1 : 0);  // the group (+ the byte after the read)
                const int sh = s0 & 3;
                u32 d[5];
                if ((s0 & ~3) + 20 <= kFqStage) {
                    const u32* lw = (const u32*)(txt + (s0 & ~3));
#pragma unroll
                    for (int i = 0; i < 5; i++) d[i] = lw[i];
                } else {
                    // past the staged bytes: global dwords holding a byte of [s0, s0 + need) below n
                    const long long gq = hrel + s0;
                    typedef __attribute__((address_space(1))) const u32 g32;
                    const g32* dw = (const g32*)((uintptr_t)(base + gq) & ~(uintptr_t)3);
#pragma unroll
                    for (int i = 0; i < 5; i++) {
                        const long long first = gq - sh + 4 * i;  // block offset of dword i
                        d[i] = (4 * i < sh + need && first < (long long)n) ? dw[i] : 0u;
                    }
                }
                const u32 x0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
                const u32 x1 = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
                const u32 x2 = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
                const u32 x3 = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
                u32 bad;
                const u32 cw = swar_group(x0, x1, x2, x3, nb, &bad);
                if constexpr (!VAR) {
                    // a newline is a non-ACGT byte: the exact test only for such groups
                    bool wrong = bad != 0u &&
                                 (has_nl(x0, nb) || has_nl(x1, nb - 4) || has_nl(x2, nb - 8) || has_nl(x3, nb - 12));
                    if (lastg) {
                        const int e = sh + nb;  // the byte after the read, in d
                        const u32 nxt = (d[e >> 2] >> (8 * (e & 3))) & 255u;
                        wrong = wrong || nxt != (u32)'\n' || hrel + s0 + nb >= (long long)n;
                    }
                    if (wrong) err |= ERR_FQ_SEQ_LEN;
                    if (bad != 0u) vhole = true;  // (ST_VHOLE: key 0's presence for padded / one-pass rows)
                } else {
                    if (bad != 0u && lr >= k) vhole = true;
                    bad |= ((1u << (16 - nb)) - 1u) & ~((1u << (16 - nb0)) - 1u);  // the slot past the read
                }
                hcodes[item] = cw;
                hinval[item] = (unsigned short)bad;
                if (SP && g == 0) rlen[rowoff + rec0 + r] = (unsigned short)L;
            };
            if constexpr (!VAR) {
                // fixed L: the groups before a read's last hold 16 bases each
                // (their loop has no byte masks and no end-of-read test), the
                // last group L - 16 (G - 1) and the byte after the read
#pragma unroll 1
                for (u32 item = (u32)lane; item < nrec * (u32)(G - 1); item += 64) {
                    const u32 r = divg1.div(item);
                    encode(r, (int)(item - r * (u32)(G - 1)), 16, false);
                }
#pragma unroll 1
                for (u32 r = (u32)lane; r < nrec; r += 64) encode(r, G - 1, L - 16 * (G - 1), true);
            } else {
#pragma unroll 1
                for (u32 item = (u32)lane; item < nrec * (u32)G; item += 64) {
                    const u32 r = divg.div(item);
                    const int g = (int)(item - r * (u32)G);
                    encode(r, g, min(16, L - 16 * g), g == G - 1);
                }
            }
            if constexpr (SP) {
                if (hn == 0) {
                    // the chunk is done: its empty rows, newline count and phase
                    const u64 nrec_c = min(((run + 3) >> 2) - rbase, max_rec);
                    const u64 row0 = c * max_rec;
                    for (u64 q = nrec_c * (u64)G + (u64)lane; q < max_rec * (u64)G; q += 64) {
                        codes[row0 * (u64)G + q] = 0u;
                        inval[row0 * (u64)G + q] = (unsigned short)0xffffu;
                    }
                    for (u64 q = nrec_c + (u64)lane; q < max_rec; q += 64) rlen[row0 + q] = 0;
                    if (lane == 0) {
                        sp_cnt[c] = run - sp_phi;
                        sp_phase[c] = (unsigned char)(sp_phi | (sp_fail ? 4u : 0u));
                    }
                }
            }
            sync();
            c = cn;
            h = hn;
        }
    }
    if (err) atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)err);
    if (__ballot(vhole) && lane == 0) atomicOr((unsigned long long*)&stats[ST_VHOLE], 1ull);
    if constexpr (VAR) {
        for (int o = 32; o >= 1; o >>= 1) vwin += __shfl_xor(vwin, o);
        if (lane == 0 && vwin) atomicAdd((unsigned long long*)&stats[ST_VWIN], (unsigned long long)vwin);
    }
}

hipError_t launch_fq_encode(const uint8_t* base, uint64_t n, const uint64_t* line_base, uint64_t max_rec, int L,
                            uint32_t* codes, uint16_t* inval, uint64_t* stats, hipStream_t s) {
    if (L < 1 || L > 32767) return hipErrorInvalidValue;
    u64 nch = fq_chunks(base, n);
    const int G = groups_per_read(L);
    const int lcap = fq_encode_list_cap(L);
    if ((u64)lcap * (u64)G >= 65536) return hipErrorInvalidValue;  // FastDivU range
    const size_t lds = (size_t)kFqEncWaves * fq_encode_wave_lds(L);
    int g = (int)hmin((nch + kFqEncWaves - 1) / kFqEncWaves, 16384);
    hipLaunchKernelGGL(fq_encode_k<false>, dim3(g ? g : 1), dim3(kFqEncBlock), lds, s, base, n, nch, line_base, max_rec,
                       L, G, lcap, codes, (unsigned short*)inval, stats, (unsigned short*)nullptr, 0, (u64*)nullptr,
                       (unsigned char*)nullptr);
    return hipGetLastError();
}

// One-pass index (fq_encode_k<false, true>): rows per chunk, the largest number
// of records whose header ends in one 16 KiB chunk (records of >= 2L + 6 bytes,
// so consecutive header ends are >= 2L + 6 bytes apart)
uint64_t fq_spec_rows_per_chunk(int L) { return 1 + (kFqChunk - 1) / (2 * (u64)L + 6); }
// the phase guess reads the first 8 newlines of a chunk's first 4 KiB
bool fq_spec_ok(int L) { return L >= 1 && 4 * (2 * L + 8) <= 4096 - 2 * L; }

hipError_t launch_fq_encode_spec(const uint8_t* base, uint64_t n, int L, uint32_t* codes, uint16_t* inval,
                                 uint16_t* rlen, uint64_t* cnt, uint8_t* phase, uint64_t* stats, hipStream_t s) {
    if (!fq_spec_ok(L)) return hipErrorInvalidValue;
    u64 nch = fq_chunks(base, n);
    const int G = groups_per_read(L);
    const int lcap = fq_encode_list_cap(L);
    if ((u64)lcap * (u64)G >= 65536 || lcap < 8) return hipErrorInvalidValue;
    const size_t lds = (size_t)kFqEncWaves * fq_encode_wave_lds(L);
    int g = (int)hmin((nch + kFqEncWaves - 1) / kFqEncWaves, 16384);
    hipLaunchKernelGGL((fq_encode_k<false, true>), dim3(g ? g : 1), dim3(kFqEncBlock), lds, s, base, n, nch,
                       (const u64*)nullptr, (u64)fq_spec_rows_per_chunk(L), L, G, lcap, codes, (unsigned short*)inval,
                       stats, (unsigned short*)rlen, 0, cnt, phase);
    return hipGetLastError();
}

// The guessed phases against the scanned newline counts (line_base = their
// exclusive scan): a chunk whose phase was not found or differs sets ERR_FQ_SPEC
__global__ __launch_bounds__(kBlock) void fq_spec_verify_k(const u64* __restrict__ line_base,
                                                           const unsigned char* __restrict__ phase, u64 nch,
                                                           u64* __restrict__ stats) {
    bool bad = false;
    for (u64 c = (u64)blockIdx.x * kBlock + threadIdx.x; c < nch; c += (u64)gridDim.x * kBlock)
        bad = bad || (phase[c] & 4u) != 0u || (u32)(line_base[c] & 3u) != (u32)(phase[c] & 3u);
    if (__ballot(bad) && lane_id() == 0) atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)ERR_FQ_SPEC);
}

hipError_t launch_fq_spec_verify(const uint64_t* line_base, const uint8_t* phase, uint64_t nch, uint64_t* stats,
                                 hipStream_t s) {
    if (nch == 0) return hipSuccess;
    hipLaunchKernelGGL(fq_spec_verify_k, dim3(grid_for(nch)), dim3(kBlock), 0, s, line_base,
                       (const unsigned char*)phase, nch, stats);
    return hipGetLastError();
}

// records of >= 32 bytes per half's list; denser halves: ERR_FQ_LIST
constexpr int kFqVarListCap = kFqHalf / 32 + 2;

bool fq_encode_var_ok(int L) {
    // (list entry, group) items are split by a FastDivU over lcap * G < 2^16
    return L >= 1 && L <= 32767 && (u64)kFqVarListCap * (u64)groups_per_read(L) < 65536;
}

hipError_t launch_fq_encode_var(const uint8_t* base, uint64_t n, const uint64_t* line_base, uint64_t max_rec, int L,
                                int k, uint32_t* codes, uint16_t* inval, uint16_t* rlen, uint64_t* stats,
                                hipStream_t s) {
    if (!fq_encode_var_ok(L) || k < 1) return hipErrorInvalidValue;
    u64 nch = fq_chunks(base, n);
    const int G = groups_per_read(L);
    const int lcap = kFqVarListCap;
    const size_t wl = (size_t)kFqStage + (((size_t)lcap * 4 + 15) & ~(size_t)15);
    const size_t lds = (size_t)kFqEncWaves * wl;
    int g = (int)hmin((nch + kFqEncWaves - 1) / kFqEncWaves, 16384);
    hipLaunchKernelGGL(fq_encode_k<true>, dim3(g ? g : 1), dim3(kFqEncBlock), lds, s, base, n, nch, line_base, max_rec, L,
                       G, lcap, codes, (unsigned short*)inval, stats, (unsigned short*)rlen, k, (u64*)nullptr,
                       (unsigned char*)nullptr);
    return hipGetLastError();
}

hipError_t launch_fq_count(const uint8_t* base, uint64_t n, uint64_t* counts, hipStream_t s) {
    u64 nch = fq_chunks(base, n);
    int g = (int)hmin((nch + kFqWaves - 1) / kFqWaves, 16384);
    hipLaunchKernelGGL(fq_count_k, dim3(g ? g : 1), dim3(kBlock), 0, s, base, n, nch, counts);
    return hipGetLastError();
}

hipError_t launch_fq_emit(const uint8_t* base, uint64_t n, const uint64_t* line_base, uint64_t* seq_off,
                          uint64_t* seq_end, uint64_t max_rec, uint64_t* stats, hipStream_t s) {
    u64 nch = fq_chunks(base, n);
    int g = (int)hmin((nch + kFqWaves - 1) / kFqWaves, 16384);
    hipLaunchKernelGGL(fq_emit_k, dim3(g ? g : 1), dim3(kBlock), 0, s, base, n, nch, line_base, seq_off, seq_end,
                       max_rec, stats);
    return hipGetLastError();
}

hipError_t launch_fq_validate(const uint64_t* seq_off, const uint64_t* seq_end, uint64_t n_rec, int L,
                              uint64_t* stats, hipStream_t s, bool at_most) {
    if (n_rec == 0) return hipSuccess;
    hipLaunchKernelGGL(fq_validate_k, dim3(grid_for(n_rec)), dim3(kBlock), 0, s, seq_off, seq_end, n_rec, L, stats,
                       at_most ? 1 : 0);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Coverage sketch (engine choice): one k-mer per read and 16-base group, the
// one starting at the group (aligned to the read, not to the genome), kept
// when a hash of its first 16 bases (its first code word) falls in 2^-rb of
// the hash space; its 56-bit fingerprint (a hash of the whole k-mer) is
// appended to `out`. The sample is a function of the k-mer, so every copy of
// a sampled k-mer is kept. Reads from a genome at coverage c repeat such a
// k-mer in ~c/16 reads (a read starting at the same position mod 16), so the
// share of distinct fingerprints estimates the coverage: iid reads ~1, cfg2's
// 30x ~0.46. The k-mer's bases are taken from the 2-bit codes (first base
// highest in each u32 of 16 bases); k-mers with a not-ACGT base are skipped.
// Per aligned position a lane loads one code word and hashes it with two u32
// multiplies; only the ~2^-rb sampled lanes load the rest of the k-mer and its
// not-ACGT masks and compute the fingerprint (the earlier form hashed every
// aligned k-mer whole with 64-bit mixes: 2.9 ms at cfg2).
// ---------------------------------------------------------------------------

__device__ __forceinline__ u32 sketch_mix32(u32 h) {  // murmur3 finaliser
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

// One thread per read, every read's code row loaded at once (G u32 words,
// 8-byte aligned rows when G is even: G/2 dwordx2 loads) so a thread waits for
// one load latency per read, not one per aligned position (GC = 0: other
// row lengths, the words one by one, 64 positions at a time). The samples are
// gathered per workgroup in LDS and appended with one global atomic per
// workgroup: the earlier form took one atomic on the single output counter
// per wave that sampled anything (~2e5 same-address atomics at cfg2, which
// serialise and set the kernel's time at ~2.4 ms).
constexpr u32 kSketchBuf = 1024;  // samples a workgroup holds in LDS (~100 expected at the default rate)

template <int GC>
__global__ __launch_bounds__(kBlock) void sketch_k(const u32* __restrict__ codes, const unsigned short* __restrict__ inval,
                                                  u64 n_reads, int G, int k, int rate_bits, u64* __restrict__ out,
                                                  u64 cap, u64* __restrict__ counter) {
    __shared__ u64 sbuf[kSketchBuf];
    __shared__ u32 scnt;
    __shared__ u64 sbase;
    const int ng = (k + 15) >> 4;  // groups a k-mer spans from a group start
    const int per = G - ng + 1;    // aligned k-mers per read
    const u32 rmask = (1u << rate_bits) - 1;
    const int nb0 = min(16, k);
    const u32 keep0 = nb0 == 16 ? 0xffffffffu : ~(0xffffffffu >> (2 * nb0));
    const u32 seed = 0x9e3779b9u ^ (u32)k;
    if (threadIdx.x == 0) scnt = 0;
    __syncthreads();
    for (u64 r0 = (u64)blockIdx.x * kBlock; r0 < n_reads; r0 += (u64)gridDim.x * kBlock) {
        const u64 r = r0 + threadIdx.x;
        const bool live = r < n_reads;
        const u64 row = (live ? r : 0) * (u64)G;
        for (int g0 = 0; g0 < (GC > 0 ? 1 : per); g0 += 64) {
            // the candidates' first words: a bit per aligned position g0 + bit
            u64 cand = 0;
            if constexpr (GC > 0) {
                u32 cw[GC];
                const u64* rp = (const u64*)(codes + row);
#pragma unroll
                for (int j = 0; j < GC / 2; j++) {
                    const u64 v = __builtin_nontemporal_load(rp + j);
                    cw[2 * j] = (u32)v;
                    cw[2 * j + 1] = (u32)(v >> 32);
                }
#pragma unroll
                for (int g = 0; g < GC; g++)
                    if (g < per && live && (sketch_mix32((cw[g] & keep0) ^ seed) & rmask) == 0) cand |= 1ull << g;
            } else {
                for (int g = g0; g < min(per, g0 + 64); g++)
                    if (live && (sketch_mix32((codes[row + (u64)g] & keep0) ^ seed) & rmask) == 0)
                        cand |= 1ull << (g - g0);
            }
            // rare: the sampled k-mers whole (their words and not-ACGT masks)
            while (cand) {
                const int g = g0 + __ffsll((long long)cand) - 1;
                cand &= cand - 1;
                const u64 base = row + (u64)g;
                u64 h = 0x243f6a8885a308d3ull ^ (u64)k;
                bool ok = true;
                for (int j = 0; j < ng; j++) {
                    const int nb = min(16, k - 16 * j);  // bases of this group inside the k-mer
                    const u32 keep = nb == 16 ? 0xffffffffu : ~(0xffffffffu >> (2 * nb));
                    const unsigned short bad =
                        (unsigned short)(inval[base + j] & (nb == 16 ? 0xffffu : ~(0xffffu >> nb)));
                    ok = ok && bad == 0;
                    h = mix64(h ^ (u64)(codes[base + j] & keep) ^ ((u64)j << 40));
                }
                if (!ok) continue;
                const u32 i = atomicAdd(&scnt, 1u);
                if (i < kSketchBuf) {
                    sbuf[i] = h >> 8;
                } else {  // a full buffer: straight out (not expected at the planned rates)
                    const u64 q = atomicAdd((unsigned long long*)counter, 1ull);
                    if (q < cap) out[q] = h >> 8;
                }
            }
        }
    }
    __syncthreads();
    const u32 m = min(scnt, kSketchBuf);
    if (threadIdx.x == 0) sbase = m ? atomicAdd((unsigned long long*)counter, (unsigned long long)m) : 0ull;
    __syncthreads();
    for (u32 i = threadIdx.x; i < m; i += kBlock)
        if (sbase + i < cap) out[sbase + i] = sbuf[i];
}

hipError_t launch_sketch(const uint32_t* codes, const uint16_t* inval, uint64_t n_reads, int L, int k, int rate_bits,
                         uint64_t* out, uint64_t cap, uint64_t* counter, hipStream_t s) {
    const int G = groups_per_read(L);
    if (G <= 0 || n_reads == 0) return hipSuccess;
    // 8 workgroups per CU (the LDS sample buffers allow them), each walking
    // its share of the reads
    const int grid = grid_for(n_reads, 2048);
#define KC_SKETCH(GCV) \
    hipLaunchKernelGGL(sketch_k<GCV>, dim3(grid), dim3(kBlock), 0, s, codes, (const unsigned short*)inval, n_reads, G, \
                       k, rate_bits, out, cap, counter)
    switch (G) {  // common read lengths: the row in registers (G even: 8-byte aligned rows)
    case 2: KC_SKETCH(2); break;
    case 4: KC_SKETCH(4); break;
    case 6: KC_SKETCH(6); break;
    case 8: KC_SKETCH(8); break;
    case 10: KC_SKETCH(10); break;
    case 12: KC_SKETCH(12); break;
    case 14: KC_SKETCH(14); break;
    case 16: KC_SKETCH(16); break;
    default: KC_SKETCH(0); break;
    }
#undef KC_SKETCH
    return hipGetLastError();
}

// The sketch's distinct fingerprints: each of the min(*counter, cap) samples
// inserted into an open-addressing set of 2^set_bits slots (fingerprint + 1,
// 0 = empty; linear probing; cap <= half the slots, so every probe ends), the
// insertions that found an empty slot counted with one atomic per wave. Same
// count as sorting the samples and counting the run heads, with no host round
// trip between the sketch and the count: *counter is read on the device.
__global__ __launch_bounds__(kBlock) void sketch_distinct_k(const u64* __restrict__ fp, const u64* __restrict__ counter,
                                                            u64 cap, u64* __restrict__ set, int set_bits,
                                                            u64* __restrict__ distinct) {
    const u64 m = min(*counter, cap);
    const u64 mask = (1ull << set_bits) - 1;
    for (u64 i0 = (u64)blockIdx.x * kBlock; i0 < m; i0 += (u64)gridDim.x * kBlock) {
        const u64 i = i0 + threadIdx.x;
        bool fresh = false;
        if (i < m) {
            const u64 v = fp[i] + 1;  // fingerprints are < 2^56
            u64 slot = mix64(v) & mask;
            for (;;) {
                const u64 old = atomicCAS((unsigned long long*)&set[slot], 0ull, (unsigned long long)v);
                if (old == 0ull) {
                    fresh = true;
                    break;
                }
                if (old == v) break;
                slot = (slot + 1) & mask;
            }
        }
        const u64 b = __ballot(fresh);
        if (lane_id() == 0 && b) atomicAdd((unsigned long long*)distinct, (unsigned long long)__popcll(b));
    }
}

hipError_t launch_sketch_distinct(const uint64_t* fp, const uint64_t* counter, uint64_t cap, uint64_t* set,
                                  int set_bits, uint64_t* distinct, hipStream_t s) {
    if (set_bits < 1 || set_bits > 40 || cap > (1ull << set_bits) / 2) return hipErrorInvalidValue;
    const int grid = grid_for(cap, 1024);
    hipLaunchKernelGGL(sketch_distinct_k, dim3(grid), dim3(kBlock), 0, s, fp, counter, cap, set, set_bits, distinct);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// synthetic FASTQ (bench/test input)
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void synth_k(kc_synth_params p, char* out) {
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < p.n; i += (u64)gridDim.x * kBlock) {
        u64 rec = p.first + i;
        if (p.layout == 1)
            kc_synth_sequence(p, rec, out + i * (u64)p.L);
        else
            kc_synth_record(p, rec, out + kc_synth_offset(p.first, rec, p.L));
    }
}

static kc_synth_params to_params(const SynthArgs& a) {
    kc_synth_params p;
    p.first = a.first;
    p.n = a.n;
    p.seed = a.seed;
    p.genome = a.genome;
    p.n_threshold = a.n_threshold;
    p.L = a.L;
    p.Lmin = a.Lmin;
    p.layout = a.layout;
    return p;
}

hipError_t launch_synth(const SynthArgs& a, char* out, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_k, dim3(grid_for(a.n, 16384)), dim3(kBlock), 0, s, to_params(a), out);
    return hipGetLastError();
}

void synth_host(const SynthArgs& a, char* out) {
    kc_synth_params p = to_params(a);
    for (u64 i = 0; i < a.n; i++) {
        u64 rec = a.first + i;
        if (a.layout == 1)
            kc_synth_sequence(p, rec, out + i * (u64)a.L);
        else
            kc_synth_record(p, rec, out + kc_synth_offset(a.first, rec, a.L));
    }
}

uint64_t synth_bytes(uint64_t first, uint64_t n, int64_t L, int layout) {
    return layout == 1 ? n * (uint64_t)L : kc_synth_offset(first, first + n, L);
}

// super-k-mer engine (F, rp_*, count_skm): see kc_skm.inl
#include "kc_skm.inl"

}  // namespace kc
