// kc_skm.inl — kernels of the super-k-mer engine ("skm"). Included by
// kc_kernels.hip inside namespace kc: it shares that file's wave helpers, the
// LDS hash insert, the global-table fallback and the P3 scan kernels.
//
// The partition engine moves every k-mer through HBM as an 8W-byte key three
// times (P2 write, P3 read + write, P5 read). Consecutive windows of a read
// share most of their bases, so the skm engine moves runs of them instead:
// a super-k-mer is a maximal run of consecutive live windows of one read whose
// minimizer bucket is equal, stored once as its bases (~1.5 B per k-mer at
// k=31 instead of 8). Per batch of reads:
//   E   encode_reads_k (shared)   reads -> 2-bit codes + not-ACGT masks
//   F   skm_front_k<W>            windows -> minimizer bucket -> records
//   S1  rp_upsweep_k/rp_scatter_k records by bucket bits 0..7  (+ digit bytes)
//   S2  rp_upsweep_k/rp_scatter_k records by bucket bits 8..15, stable over
//                                 S1's regions -> grouped by bucket
//   P4  bucket_bounds_k (shared)  bucket ranges
//   P5  count_skm_k<W>            per bucket: expand records into keys, count
//                                 in the LDS table (sub-range passes, global
//                                 table and spill exactly as count_buckets)
// Finish: the (key, count) records are grouped by their first 8 bases with
// the same rp_* passes (counts as payload) and every group is sorted in LDS
// by seg_sort_k, so the output needs no global sort.
//
// Bucket of a window: the minimum over the window's m-mers (its first k bases,
// all ACGT for a live window) of mmer_hash, low 16 bits. It is a function of
// the key, so equal keys always meet in one bucket; counts stay exact for any
// input (the bucket only decides where a key is counted).
//
// Record (RW = W + 1 u64 words, SoA): the words concatenated MSB-first hold
//   bits [0, 16)          bucket (so word0 >> 48 is the bucket: the rp_*
//                         passes and bucket_bounds_k read it like a key prefix)
//   bits [16, 16 + 2 nb)  nb = K' + n - 1 bases, 2 bits each (A0 C1 G2 T3,
//                         other bytes 3, bases past the read end 0), where K'
//                         is the key span (k when the last key word is masked,
//                         32W otherwise: GPUHandler.cu:181-186)
//   low 6 bits            n, the number of keys (0 = padding record, bucket
//                         0xffff, which no window is given)
// Key i of the record = K' bases from base i (the window i positions after
// the run start) = exactly the key extractKMers builds for that window.
// nb <= 32 RW - 11, so n <= nmax = 32 RW - 10 - K'; longer runs are split.

constexpr int kSkmBlock = 256;
constexpr int kSkmPf = 2;  // F: code words prefetched per thread
constexpr int kSkmHq = 22;  // F: most m-mer positions per hash item

__device__ __forceinline__ u32 fmix32(u32 x) {
    x ^= x >> 16;
    x *= 0x85ebca6bu;
    x ^= x >> 13;
    x *= 0xc2b2ae35u;
    x ^= x >> 16;
    return x;
}

// m-mer order: m <= 12 uses a 24-bit multiplicative hash of the m-mer (full
// rate), m <= 16 a 32-bit one; either way the low 16 bits (the bucket) are a
// bijection of its last 8 bases. Longer m-mers are folded to 32 bits first.
__device__ __forceinline__ u32 mmer_hash(u64 mm) {
    const u32 x = (u32)mm ^ ((u32)(mm >> 32) * 0x9e3779b1u);
    return (x ^ 0x5bd1e995u) * 0x9e3779b1u;
}

// full-rate 24 x 24 -> low 32 bits multiply by a uniform b (the compiler
// keeps v_mul_lo_u32)
__device__ __forceinline__ u32 mul_u24(u32 a, u32 b) {
    u32 r;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "s"(b), "v"(a));
    return r;
}

__device__ __forceinline__ u64 readlane64(u64 v, int l) {
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)v, l);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), l);
    return ((u64)hi << 32) | lo;
}

struct SkmArgs {
    const u32* codes;             // kernel E output, G u32 per read
    const unsigned short* inval;  //   not-ACGT masks, G u16 per read
    int G;
    u64 n_reads;
    int L, k, m, Kp, nmax, R, NG, HS;
    int hq;     // m-mer positions per hash item
    u64 chunk;  // pool records per wave allocation (>= records of one tile)
    int skip;  // timing experiments only (KC_F_SKIP): 1 record stores, 2 runs + records, 4 minimizer, 8 hashes
    u64* pool;         // RW x pool_cap u64 (SoA)
    u64 pool_cap;
    u64* pool_cursor;  // chunk allocator (records handed out)
    unsigned char* dig1;  // optional: a record's low bucket byte (the first grouping pass's digit)
    u64* stats;
};

struct SkmLds {
    size_t codes, inval, hm, wpk, rflag, sa, ea, total;
};

// LDS skew of the m-mer hashes: a lane works on 8 consecutive windows, so
// lanes read hm at a stride of 8 words; one pad word per 8 makes the stride 9
// (no bank conflicts)
__host__ __device__ inline int skm_sk(int j) { return j + (j >> 3); }
__host__ __device__ inline int skm_hsk(int HS) { return skm_sk(HS) + 1; }

// One wave's LDS region (F). wpk: 16 B per 8-window chunk (the chunk's eight
// 16-bit window buckets, 0xffff = no key); sa: run starts (window | bucket <<
// 16); ea: run ends.
__host__ __device__ inline SkmLds skm_lds_layout(int R, int NG, int HS, int nw) {
    SkmLds o;
    size_t p = 0;
    const int nchr = (nw + 7) / 8;
    o.wpk = p;
    p += (size_t)R * nchr * 16;
    o.codes = p;
    p += (size_t)R * NG * 4;
    o.inval = p;
    p += (size_t)R * NG * 4;
    o.hm = p;
    p += (size_t)R * skm_hsk(HS) * 4;
    o.rflag = p;
    p += (size_t)R * 4;
    o.sa = p;
    p += (size_t)R * nw * 4;
    o.ea = p;
    p += (size_t)R * nw * 2;
    p = (p + 15) & ~(size_t)15;
    o.total = p;
    return o;
}

// Intra-wave LDS hand-off (lane a writes, lane b reads): the fences are
// limited to LDS, so they never wait for global loads in flight (prefetch)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// Inclusive scan of one u32 per lane over the wave (Hillis-Steele).
__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(v, o);
        if (lane >= o) v += y;
    }
    return v;
}

constexpr u32 kNoKey = 0xffffu;  // window bucket of a window without a key (dead)

// F: every wave works alone on tiles of R reads (its own LDS region; no
// workgroup barriers, so the waves of a CU hide each other's latency):
//   1. code words and masks of the tile into LDS (prefetched into registers
//      during the previous tile; groups past the read stay zero); per read:
//      bit 0 = a base outside ACGT, bit 1 = an 8-base aligned all-A group
//      (only such reads can hold a key 0^W: a key spans >= 18 real bases)
//   2. hm[r][j] = mmer_hash of the m bases from j (hq positions per lane)
//   3. per 8-window chunk: window minimum over its k-m+1 m-mers as
//      min(left suffix, shared core, right prefix); reads with a flag take
//      the rolling-key check of count_front (valid, key != 0); the chunk's
//      eight buckets (kNoKey: no key) packed into 16 bytes
//   4. run starts (bucket differs from the previous window's) and ends from
//      the packed buckets of the chunk and its two neighbours, compacted in
//      tile order by a wave scan: the i-th start pairs with the i-th end
//   5. runs -> pieces of <= nmax windows -> records at consecutive positions
//      of the wave's current pool chunk (one global atomic per chunk); the
//      chunk tail is padded with n = 0 records at exit
template <int W>
#ifndef KC_F_WPE
#define KC_F_WPE 5  // F: waves per SIMD the register budget is cut for
#endif
__global__ __launch_bounds__(kSkmBlock) __attribute__((amdgpu_waves_per_eu(KC_F_WPE, 8))) void skm_front_k(SkmArgs a) {
    constexpr int RW = W + 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int L = a.L, k = a.k, m = a.m, NG = a.NG, HS = a.HS, R = a.R, Kp = a.Kp, G = a.G;
    const u32 nmax = (u32)a.nmax;
    const int nw = L - k + 1;
    const int wm = k - m + 1;  // m-mers per window (>= 8)
    const int nchr = (nw + 7) >> 3;
    const int hq = a.hq;
    const int hch = (HS + hq - 1) / hq;
    const int HSK = skm_hsk(hch * hq);  // hash items cover hch * hq positions
    const FastDivU div_nchr((u32)nchr), div_hch((u32)hch), div_nw((u32)nw), div_g((u32)G);
    const SkmLds lay = skm_lds_layout(R, NG, hch * hq, nw);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    unsigned char* wb = smem + (size_t)wave * lay.total;
    u32* codes = (u32*)(wb + lay.codes);
    u32* inval = (u32*)(wb + lay.inval);
    u32* hm = (u32*)(wb + lay.hm);
    v4u* wpk = (v4u*)(wb + lay.wpk);
    u32* rflag = (u32*)(wb + lay.rflag);
    u32* sa = (u32*)(wb + lay.sa);
    unsigned short* ea = (unsigned short*)(wb + lay.ea);
    const bool mask_last = ((k + 3) / 4) < 8 * W;
    const u64 last_mask = mask_last ? (~0ull << (64 - 2 * (k & 31))) : ~0ull;
    const u64 ntiles = (a.n_reads + R - 1) / R;
    const u64 wid = (u64)blockIdx.x * (kSkmBlock / 64) + wave;
    const u64 nwaves = (u64)gridDim.x * (kSkmBlock / 64);
    const u64 chunk = a.chunk;
    const bool m16 = m <= 16, m12 = m <= 12;
    u64 my_valid = 0;
    bool my_hole = false;
    for (int it = lane; it < R * NG; it += 64) {
        codes[it] = 0;
        inval[it] = 0;
    }
    int pr[kSkmPf], pg[kSkmPf];
#pragma unroll
    for (int j = 0; j < kSkmPf; j++) {
        const int it = lane + j * 64;
        pr[j] = it / G;
        pg[j] = it - pr[j] * G;
    }
    u32 pfc[kSkmPf], pfi[kSkmPf];
    auto prefetch = [&](u64 tile) {
        const u64 r0 = tile * (u64)R;
        const int nr = tile < ntiles ? (int)min((u64)R, a.n_reads - r0) : 0;
#pragma unroll
        for (int j = 0; j < kSkmPf; j++) {
            u32 cw = 0, iv = 0;
            if (pr[j] < nr) {
                const u64 idx = (r0 + (u64)pr[j]) * (u64)G + (u64)pg[j];
                cw = __builtin_nontemporal_load(a.codes + idx);
                iv = __builtin_nontemporal_load(a.inval + idx);
            }
            pfc[j] = cw;
            pfi[j] = iv;
        }
    };
    auto flag_of = [&](u32 cw, u32 iv, int g) -> u32 {
        // aligned all-A halves inside the read (a key 0^W has >= k >= 18 A
        // bases of the read in a row, so it holds one; halves with padding
        // past L would flag every read whose L is not a multiple of 8)
        const bool za = g < G && (((cw >> 16) == 0u && 16 * g + 8 <= a.L) || ((cw & 0xffffu) == 0u && 16 * g + 16 <= a.L));
        return (iv ? 1u : 0u) | (za ? 2u : 0u);
    };
    prefetch(wid);
    u64 ccur = 0, cend = 0;  // the wave's pool chunk (wave-uniform)
    wave_sync();
    for (u64 tile = wid; tile < ntiles; tile += nwaves) {
        const u64 r0 = tile * (u64)R;
        const int nr = (int)min((u64)R, a.n_reads - r0);
        // 1. codes and read flags
        for (int r = lane; r < nr; r += 64) rflag[r] = 0;
        wave_sync();
#pragma unroll
        for (int j = 0; j < kSkmPf; j++)
            if (pr[j] < nr) {
                codes[pr[j] * NG + pg[j]] = pfc[j];
                inval[pr[j] * NG + pg[j]] = pfi[j];
                const u32 f = flag_of(pfc[j], pfi[j], pg[j]);
                if (f) atomicOr(&rflag[pr[j]], f);
            }
        for (int it = lane + kSkmPf * 64; it < nr * G; it += 64) {
            const int r = (int)div_g.div((u32)it), g = it - r * G;
            const u64 idx = (r0 + (u64)r) * (u64)G + (u64)g;
            const u32 cw = a.codes[idx], iv = a.inval[idx];
            codes[r * NG + g] = cw;
            inval[r * NG + g] = iv;
            const u32 f = flag_of(cw, iv, g);
            if (f) atomicOr(&rflag[r], f);
        }
        wave_sync();
        prefetch(tile + nwaves);
        // 2. m-mer hashes (positions past L - m are never used by a window)
        for (int it = lane; it < ((a.skip & 8) ? 0 : nr * hch); it += 64) {
            const int r = (int)div_hch.div((u32)it), j0 = (it - r * hch) * hq;
            const u64 x = code_word(codes + r * NG, j0);
            u32* hr = hm + r * HSK;
            if (m12) {
                // m <= 12: the m-mer fits 24 bits, so the full-rate 24-bit
                // multiply orders it (odd constant: a bijection)
                // (hm is padded to hch * hq positions: no bound check)
                u64 xs = x;
                for (int i = 0; i < hq; i++) {
                    const u32 mm = (u32)(xs >> (64 - 2 * m));
                    hr[skm_sk(j0 + i)] = mul_u24(mm ^ 0xd1e995u, 0x9e3779u);
                    xs <<= 2;
                }
            } else if (m16) {
                const u32 xh = (u32)(x >> 32), xl = (u32)x;
                for (int i = 0; i < hq; i++) {
                    const u32 w = i == 0 ? xh : (i < 16 ? __builtin_amdgcn_alignbit(xh, xl, 32 - 2 * i) : xl << (2 * i - 32));
                    const u32 mm = w >> (32 - 2 * m);
                    if (j0 + i < HS) hr[skm_sk(j0 + i)] = (mm ^ 0x5bd1e995u) * 0x9e3779b1u;
                }
            } else {
                for (int i = 0; i < hq; i++)
                    if (j0 + i < HS) hr[skm_sk(j0 + i)] = mmer_hash((x << (2 * i)) >> (64 - 2 * m));
            }
        }
        wave_sync();
        // 3. windows -> packed chunk buckets
        for (int c = lane; c < nr * nchr; c += 64) {
            const int r = (int)div_nchr.div((u32)c), p0 = (c - r * nchr) * 8;
            const u32* hr = hm + r * HSK;
            const int h0 = 9 * (p0 >> 3);  // skm_sk(p0 + i) = h0 + i for i < 8
            u32 core = ~0u;
            const int jl = p0 + wm - 1;
            for (int jb = p0 + 7; jb <= ((a.skip & 4) ? -1 : jl); jb += 8) {
                u32 v8[8];
#pragma unroll
                for (int i = 0; i < 8; i++) v8[i] = hr[skm_sk(min(jb + i, jl))];
#pragma unroll
                for (int i = 0; i < 8; i++) core = min(core, v8[i]);
            }
            u32 lft[8];
            lft[7] = ~0u;
#pragma unroll
            for (int i = 6; i >= 0; i--) lft[i] = min(lft[i + 1], hr[h0 + i]);
            u32 rgt = ~0u;
            u32 bk[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (i > 0) rgt = min(rgt, hr[skm_sk(jl + i)]);
                u32 b = min(core, min(lft[i], rgt)) & 0xffffu;
                bk[i] = b == kNoKey ? kNoKey - 1u : b;
            }
            const u32 fl = rflag[r];
            u32 act = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) act += (p0 + i < nw) ? 1u : 0u;
            if (fl == 0u) {
                my_valid += act;
            } else {
                // invalid bases or a possible key 0^W: the rolling key check
                const u32* cr = codes + r * NG;
                u64 kr[W];
#pragma unroll
                for (int j = 0; j < W; j++) kr[j] = code_word(cr, p0 + 32 * j);
                u64 tl = code_word(cr, p0 + 32 * W);
                u32 zeros = 0, valids = 0;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int p = p0 + i;
                    const bool active = p < nw;
                    bool valid = active;
                    if (active && (fl & 1u)) {
                        const u32* ir = inval + r * NG;
                        const int last = p + k - 1;
                        for (int gg = p >> 4; gg <= (last >> 4); gg++) {
                            const int lo = max(p - 16 * gg, 0), hi = min(last - 16 * gg, 15);
                            const u32 rm = (0xffffu >> lo) & (0xffffu << (15 - hi)) & 0xffffu;
                            if (ir[gg] & rm) valid = false;
                        }
                    }
                    bool is_zero = (kr[W - 1] & last_mask) == 0ull;
#pragma unroll
                    for (int j = 0; j < W - 1; j++) is_zero = is_zero && (kr[j] == 0ull);
                    my_hole |= active && !valid;
                    valids += valid ? 1u : 0u;
                    zeros += (valid && is_zero) ? 1u : 0u;
                    if (!valid || is_zero) bk[i] = kNoKey;
#pragma unroll
                    for (int j = 0; j < W - 1; j++) kr[j] = (kr[j] << 2) | (kr[j + 1] >> 62);
                    kr[W - 1] = (kr[W - 1] << 2) | (tl >> 62);
                    tl <<= 2;
                }
                my_valid += valids;
                if (zeros) {
                    atomicAdd((unsigned long long*)&a.stats[ST_KEY0], (unsigned long long)zeros);
                    atomicOr((unsigned long long*)&a.stats[ST_KEY0_PRESENT], 1ull);
                }
            }
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (p0 + i >= nw) bk[i] = kNoKey;
            v4u pk;
            pk.x = bk[0] | (bk[1] << 16);
            pk.y = bk[2] | (bk[3] << 16);
            pk.z = bk[4] | (bk[5] << 16);
            pk.w = bk[6] | (bk[7] << 16);
            wpk[c] = pk;
        }
        wave_sync();
        if (a.skip & 2) continue;
        // 4. run starts / ends, compacted in tile order
        u32 sbase = 0, ebase = 0;
        for (int c0 = 0; c0 < nr * nchr; c0 += 64) {
            const int c = c0 + lane;
            u32 smask = 0, emask = 0;
            int q0 = 0;
            u32 bk[8];
            v4u pkv;
            if (c < nr * nchr) {
                const int r = (int)div_nchr.div((u32)c), p0 = (c - r * nchr) * 8;
                q0 = r * nw + p0;
                const v4u pk = wpk[c];
                pkv = pk;
                bk[0] = pk.x & 0xffffu;
                bk[1] = pk.x >> 16;
                bk[2] = pk.y & 0xffffu;
                bk[3] = pk.y >> 16;
                bk[4] = pk.z & 0xffffu;
                bk[5] = pk.z >> 16;
                bk[6] = pk.w & 0xffffu;
                bk[7] = pk.w >> 16;
                u32 prev = p0 > 0 ? (wpk[c - 1].w >> 16) : kNoKey;
                const u32 nx8 = p0 + 8 < nw ? (wpk[c + 1].x & 0xffffu) : kNoKey;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const u32 v = bk[i];
                    const u32 nx = i < 7 ? bk[i + 1] : nx8;
                    if (v != kNoKey) {
                        if (v != prev) smask |= 1u << i;
                        if (v != nx) emask |= 1u << i;
                    }
                    prev = v;
                }
            }
            const u32 v = (u32)__popc(smask) | ((u32)__popc(emask) << 16);
            const u32 inc = wave_incl_scan(v);
            const u32 ex = inc - v;
            const u32 tot = (u32)__builtin_amdgcn_readlane((int)inc, 63);
            u32 sp = sbase + (ex & 0xffffu), ep = ebase + (ex >> 16);
            // set bits only (a lane holds one or two starts and ends)
            for (u32 mm = smask; mm; mm &= mm - 1u) {
                const int i = __builtin_ctz(mm);
                const u32 wv = (i & 4) ? ((i & 2) ? pkv.w : pkv.z) : ((i & 2) ? pkv.y : pkv.x);
                sa[sp++] = (u32)(q0 + i) | (((wv >> (16 * (i & 1))) & 0xffffu) << 16);
            }
            for (u32 mm = emask; mm; mm &= mm - 1u) ea[ep++] = (unsigned short)(q0 + __builtin_ctz(mm));
            sbase += tot & 0xffffu;
            ebase += tot >> 16;
        }
        wave_sync();
        // 5. runs -> records
        const u32 T = sbase;
        const u32 per = (T + 63) >> 6;
        const u32 i0 = min(T, (u32)lane * per), i1 = min(T, i0 + per);
        u32 mine = 0;
        for (u32 i = i0; i < i1; i++) {
            const u32 n = (u32)ea[i] - (sa[i] & 0xffffu) + 1u;
            mine += n <= nmax ? 1u : (n + nmax - 1) / nmax;
        }
        const u32 pinc = wave_incl_scan(mine);
        const u32 pb = pinc - mine;
        const u32 ptot = (u32)__builtin_amdgcn_readlane((int)pinc, 63);
        const u64 room = cend - ccur;
        const u64 oc = ccur;
        u64 nbase = 0;
        if ((u64)ptot > room) {
            u64 nb = 0;
            if (lane == 0) nb = atomicAdd((unsigned long long*)a.pool_cursor, (unsigned long long)chunk);
            nb = readlane64(nb, 0);
            nbase = nb;
            ccur = nb + ((u64)ptot - room);
            cend = nb + chunk;
        } else {
            ccur += ptot;
        }
        u32 g = pb;
        for (u32 i = i0; i < i1; i++) {
            const u32 sv = sa[i];
            const u32 qs = sv & 0xffffu;
            const u32 n = (u32)ea[i] - qs + 1u;
            const int r = (int)div_nw.div(qs);
            const int ps0 = (int)qs - r * nw;
            const u64 bkt = sv >> 16;
            const u32* cr = codes + r * NG;
            for (u32 off = 0; off < n; off += nmax, g++) {
                const u32 nn = min(nmax, n - off);
                const int ps = ps0 + (int)off;
                u64 rec[RW];
                rec[0] = (bkt << 48) | (code_word(cr, ps) >> 16);
#pragma unroll
                for (int j = 1; j < RW; j++) rec[j] = code_word(cr, ps + 32 * j - 8);
                const int vb = 16 + 2 * (Kp + (int)nn - 1);
#pragma unroll
                for (int j = 0; j < RW; j++) {
                    const int bits = vb - 64 * j;
                    const u64 msk = bits >= 64 ? ~0ull : (bits <= 0 ? 0ull : (~0ull << (64 - bits)));
                    rec[j] &= msk;
                }
                rec[RW - 1] |= (u64)nn;
                const u64 dst = (u64)g < room ? oc + g : nbase + ((u64)g - room);
                if (dst < a.pool_cap && !(a.skip & 1)) {
#pragma unroll
                    for (int j = 0; j < RW; j++) a.pool[(u64)j * a.pool_cap + dst] = rec[j];
                    if (a.dig1) a.dig1[dst] = (unsigned char)bkt;
                }
            }
        }
        wave_sync();
    }
    // pad the rest of the wave's chunk with n = 0 records in bucket kNoKey,
    // which no window takes: P5 never walks them
    for (u64 i = ccur + (u64)lane; i < cend; i += 64)
        if (i < a.pool_cap) {
#pragma unroll
            for (int j = 0; j < RW; j++) a.pool[(u64)j * a.pool_cap + i] = j == 0 ? ((u64)kNoKey << 48) : 0ull;
            if (a.dig1) a.dig1[i] = (unsigned char)kNoKey;
        }
    wave_add(&a.stats[ST_VALID], my_valid);
    if (__ballot(my_hole) && lane == 0) atomicOr((unsigned long long*)&a.stats[ST_KEY0_PRESENT], 1ull);
}

// ---------------------------------------------------------------------------
// F2: skm_front2_k<W, K>, F for a compile-time k whose minimizer length is 11
// (every k of W = 1; skm_geometry picks m = 11 there). Same records, buckets
// and statistics as skm_front_k; what changes is the instruction count:
//   - k, K', nmax, m and the window span are constants: the m-mers of a hash
//     item (16 positions of one code-word pair) are extracted with immediate
//     shifts, written two per LDS store at immediate offsets, and a chunk's
//     k - m + 8 hashes are read at immediate offsets into registers
//   - the chunk's eight buckets stay in registers; the neighbouring chunks'
//     first / last bucket come from the neighbouring lanes (wave shuffles)
//   - the tile's start / end counts are scanned by ballots of their bits
//     (counts <= 8), and the ends' positions follow from the starts' (a run
//     open across a chunk boundary is the only difference)
//   - every lane's roles (prefetch item, hash item, chunk) are fixed for the
//     kernel (divisions once), record words are assembled branch-free
// Requirements (launch_skm_front checks them): ceil((L - k + 1) / 8) <= 64.
// ---------------------------------------------------------------------------

template <int W, int K>
struct F2Cfg {
    static constexpr int RW = W + 1;
    static constexpr bool MASK = ((K + 3) / 4) < 8 * W;
    static constexpr int KP = MASK ? K : 32 * W;
    static constexpr int NMAX0 = 32 * RW - 10 - KP;
    static constexpr int NMAX = NMAX0 > 63 ? 63 : NMAX0;
    static constexpr int M = 11;
    static constexpr int WM = K - M + 1;  // m-mers per window
    static constexpr u64 LAST_MASK = MASK ? (~0ull << (64 - 2 * (K & 31))) : ~0ull;
    static_assert(WM >= 8, "a window spans at least 8 m-mers");
};

struct F2Args {
    const u32* codes;             // kernel E output, G u32 per read
    const unsigned short* inval;  //   not-ACGT masks, G u16 per read
    u64 n_reads, ntiles;
    int G, nw, nchr, R, NG, NI, HSK;
    u32 o_inval, o_hm, o_rflag, o_sa, o_ea, o_bk, wbytes;  // a wave's LDS region (bytes)
    u64 chunk;  // pool records per wave allocation (>= records of one tile)
    u64* pool;
    u64 pool_cap;
    u64* pool_cursor;
    unsigned char* dig1;
    u64* stats;
    int skip;  // timing experiments only (KC_F_SKIP): 1 record stores, 2 runs + records, 4 window minima, 8 hashes
};

constexpr int kF2Pf = 2;  // F2: code words prefetched per lane

// 22-bit m-mer (m = 11) at base i of the 32 bases {c0, c1} (MSB first)
template <int I>
__device__ __forceinline__ u32 f2_mmer(u32 c0, u32 c1) {
    if constexpr (I <= 5)
        return (c0 >> (10 - 2 * I)) & 0x3fffffu;
    else
        return __builtin_amdgcn_alignbit(c0, c1, 42 - 2 * I) & 0x3fffffu;
}

template <int I>
__device__ __forceinline__ void f2_hash_pair(u32* hp, u32 c0, u32 c1) {
    // hp[sk(i)]: positions 2j, 2j + 1 of an 8-group are adjacent words
    const u32 h0 = mul_u24(f2_mmer<I>(c0, c1) ^ 0xd1e995u, 0x9e3779u);
    const u32 h1 = mul_u24(f2_mmer<I + 1>(c0, c1) ^ 0xd1e995u, 0x9e3779u);
    hp[I + (I >> 3)] = h0;
    hp[I + 1 + (I >> 3)] = h1;
}

// 64 bits from base b of a code row (MSB first), branch-free
__device__ __forceinline__ u64 f2_code_word(const u32* cr, int b) {
    const int g = b >> 4, o = b & 15;
    const u32 c0 = cr[g], c1 = cr[g + 1], c2 = cr[g + 2];
    const u32 hi = o ? __builtin_amdgcn_alignbit(c0, c1, 32 - 2 * o) : c0;
    const u32 lo = o ? __builtin_amdgcn_alignbit(c1, c2, 32 - 2 * o) : c1;
    return ((u64)hi << 32) | lo;
}

// exclusive prefix over the wave of v < 16 (4 bit-plane ballots); *tot = sum
__device__ __forceinline__ u32 f2_scan16(u32 v, u32* tot) {
    const u64 lt = lanemask_lt();
    u32 ex = 0, t = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const u64 bl = __ballot((v >> b) & 1u);
        ex += (u32)__popcll(bl & lt) << b;
        t += (u32)__popcll(bl) << b;
    }
    *tot = t;
    return ex;
}

template <int W, int K>
__global__ __launch_bounds__(kSkmBlock) __attribute__((amdgpu_waves_per_eu(KC_F_WPE, 8))) void skm_front2_k(F2Args a) {
    using C = F2Cfg<W, K>;
    constexpr int RW = C::RW;
    constexpr int WM = C::WM;
    constexpr u32 NMAX = (u32)C::NMAX;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    unsigned char* wb = smem + (size_t)wave * a.wbytes;
    u32* codes = (u32*)wb;
    u32* inval = (u32*)(wb + a.o_inval);
    u32* hm = (u32*)(wb + a.o_hm);
    u32* rflag = (u32*)(wb + a.o_rflag);
    unsigned short* sa = (unsigned short*)(wb + a.o_sa);  // run starts (tile window index)
    unsigned short* ea = (unsigned short*)(wb + a.o_ea);  // run ends
    unsigned short* wbk = (unsigned short*)(wb + a.o_bk);  // window buckets, 8 per lane (chunk)
    const int G = a.G, NG = a.NG, R = a.R, nw = a.nw, nchr = a.nchr, NI = a.NI, HSK = a.HSK;
    const int L = nw + K - 1;
    const int RG = R * G;
    const u64 wid = (u64)blockIdx.x * (kSkmBlock / 64) + wave;
    const u64 nwaves = (u64)gridDim.x * (kSkmBlock / 64);
    for (int it = lane; it < R * NG; it += 64) {
        codes[it] = 0;
        inval[it] = 0;
    }
    // fixed roles of this lane
    const FastDivU div_g((u32)G), div_ni((u32)NI), div_nw((u32)nw);
    int pr[kF2Pf], pg[kF2Pf];
#pragma unroll
    for (int j = 0; j < kF2Pf; j++) {
        const int it = lane + 64 * j;
        pr[j] = (int)div_g.div((u32)it);
        pg[j] = it - pr[j] * G;
    }
    int po[kF2Pf];  // LDS word of each prefetched code word
#pragma unroll
    for (int j = 0; j < kF2Pf; j++) po[j] = pr[j] * NG + pg[j];
    const int hr0 = (int)div_ni.div((u32)lane), hq0 = lane - hr0 * NI;  // first hash item
    const int cr_ = lane / nchr, cc = lane - (lane / nchr) * nchr;     // chunk: read, chunk of the read
    const int p0 = 8 * cc;
    // per-lane constants of the chunk: its hash row, code rows, windows
    const u32* hbase = hm + (cr_ < R ? cr_ : 0) * HSK + 9 * cc;
    const u32* crw0 = codes + (cr_ < R ? cr_ : 0) * NG;
    const u32* irw0 = inval + (cr_ < R ? cr_ : 0) * NG;
    const u32 act = (u32)max(0, min(8, nw - p0));
    const u32 actm = (1u << act) - 1u;  // the chunk's windows inside the read
    const u32 q0 = (u32)(cr_ * nw + p0);
    const bool first_chunk = cc == 0, last_chunk = cc == nchr - 1;
    u32 pfc[kF2Pf], pfi[kF2Pf];
    auto prefetch = [&](u64 tile) {
        const u64 r0 = tile * (u64)R;
        const int nr = tile < a.ntiles ? (int)min((u64)R, a.n_reads - r0) : 0;
        const u64 base = tile * (u64)RG;
#pragma unroll
        for (int j = 0; j < kF2Pf; j++) {
            u32 cw = 0, iv = 0;
            if (pr[j] < nr) {
                cw = __builtin_nontemporal_load(a.codes + base + (u64)(lane + 64 * j));
                iv = __builtin_nontemporal_load(a.inval + base + (u64)(lane + 64 * j));
            }
            pfc[j] = cw;
            pfi[j] = iv;
        }
    };
    auto flag_of = [&](u32 cw, u32 iv, int g) -> u32 {
        // non-ACGT bases; aligned all-A halves inside the read (a key 0^W
        // has >= k A bases of the read in a row): only such reads can hold
        // a key 0^W
        const bool za = g < G && (((cw >> 16) == 0u && 16 * g + 8 <= L) || ((cw & 0xffffu) == 0u && 16 * g + 16 <= L));
        return (iv ? 1u : 0u) | (za ? 2u : 0u);
    };
    prefetch(wid);
    u64 my_valid = 0;
    bool my_hole = false;
    u64 ccur = 0, cend = 0;  // the wave's pool chunk (wave-uniform)
    wave_sync();
    for (u64 tile = wid; tile < a.ntiles; tile += nwaves) {
        const u64 r0 = tile * (u64)R;
        const int nr = (int)min((u64)R, a.n_reads - r0);
        // 1. code words, masks and read flags into LDS
        if (lane < nr) rflag[lane] = 0;
        wave_sync();
#pragma unroll
        for (int j = 0; j < kF2Pf; j++)
            if (pr[j] < nr) {
                codes[po[j]] = pfc[j];
                inval[po[j]] = pfi[j];
                const u32 f = flag_of(pfc[j], pfi[j], pg[j]);
                if (f) atomicOr(&rflag[pr[j]], f);
            }
        for (int it = lane + kF2Pf * 64; it < nr * G; it += 64) {
            const int r = (int)div_g.div((u32)it), g = it - r * G;
            const u64 idx = tile * (u64)RG + (u64)it;
            const u32 cw = a.codes[idx], iv = a.inval[idx];
            codes[r * NG + g] = cw;
            inval[r * NG + g] = iv;
            const u32 f = flag_of(cw, iv, g);
            if (f) atomicOr(&rflag[r], f);
        }
        wave_sync();
        prefetch(tile + nwaves);
        // 2. m-mer hashes, 16 positions per item
        for (int it2 = lane; it2 < ((a.skip & 8) ? 0 : nr * NI); it2 += 64) {
            int hr = hr0, hq = hq0;
            if (it2 != lane) {
                hr = (int)div_ni.div((u32)it2);
                hq = it2 - hr * NI;
            }
            const u32* crow = codes + hr * NG + hq;
            const u32 c0 = crow[0], c1 = crow[1];
            u32* hp = hm + hr * HSK + 18 * hq;
            f2_hash_pair<0>(hp, c0, c1);
            f2_hash_pair<2>(hp, c0, c1);
            f2_hash_pair<4>(hp, c0, c1);
            f2_hash_pair<6>(hp, c0, c1);
            f2_hash_pair<8>(hp, c0, c1);
            f2_hash_pair<10>(hp, c0, c1);
            f2_hash_pair<12>(hp, c0, c1);
            f2_hash_pair<14>(hp, c0, c1);
        }
        wave_sync();
        // 3. this lane's chunk: eight window buckets (kNoKey: no key)
        const bool live_lane = lane < nr * nchr;
        u32 bk[8];
        {
            const u32* hb = hbase;
            u32 h[WM + 7];
#pragma unroll
            for (int j = 0; j < WM + 7; j++) h[j] = hb[j + (j >> 3)];
            u32 core = h[7];
            if (!(a.skip & 4))
#pragma unroll
                for (int j = 8; j < WM; j++) core = min(core, h[j]);
            u32 lf[8];
            lf[7] = ~0u;
#pragma unroll
            for (int i = 6; i >= 0; i--) lf[i] = min(lf[i + 1], h[i]);
            u32 rt = ~0u;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (i > 0) rt = min(rt, h[WM - 1 + i]);
                const u32 b = min(core, min(lf[i], rt)) & 0xffffu;
                bk[i] = min(b, kNoKey - 1u);
            }
        }
        u32 livem = live_lane ? actm : 0u;  // windows that keep their bucket
        if (live_lane) {
            const u32 fl = rflag[cr_];
            if (fl == 0u) {
                my_valid += act;
            } else {
                // invalid bases (flag 1): a window is dead when one of its K
                // bases is not ACGT (not-ACGT bits of bases p0 .. p0 + 55 in
                // one 64-bit word); a possible key 0^W (flag 2): rolling keys
                const u32* crw = crw0;
                const u32* ir = irw0;
                u32 badm = 0;
                if (fl & 1u) {
                    const int g0 = p0 >> 4;
                    const u64 X = (((u64)ir[g0] << 48) | ((u64)ir[g0 + 1] << 32) | ((u64)ir[g0 + 2] << 16) |
                                   (u64)ir[g0 + 3])
                                  << (p0 & 15);
                    constexpr u64 KM = ~0ull << (64 - K);  // a window's K bases
#pragma unroll
                    for (int i = 0; i < 8; i++) badm |= ((X & (KM >> i)) ? 1u : 0u) << i;
                }
                u32 zm = 0;
                if (fl & 2u) {
                    u64 kr[W];
#pragma unroll
                    for (int j = 0; j < W; j++) kr[j] = f2_code_word(crw, p0 + 32 * j);
                    u64 tl = f2_code_word(crw, p0 + 32 * W);
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        bool is_zero = (kr[W - 1] & C::LAST_MASK) == 0ull;
#pragma unroll
                        for (int j = 0; j < W - 1; j++) is_zero = is_zero && (kr[j] == 0ull);
                        zm |= (is_zero ? 1u : 0u) << i;
#pragma unroll
                        for (int j = 0; j < W - 1; j++) kr[j] = (kr[j] << 2) | (kr[j + 1] >> 62);
                        kr[W - 1] = (kr[W - 1] << 2) | (tl >> 62);
                        tl <<= 2;
                    }
                }
                const u32 validm = actm & ~badm;
                const u32 zeros = (u32)__popc(validm & zm);
                my_hole |= (actm & badm) != 0u;
                my_valid += (u32)__popc(validm);
                livem = validm & ~zm;
                if (zeros) {
                    atomicAdd((unsigned long long*)&a.stats[ST_KEY0], (unsigned long long)zeros);
                    atomicOr((unsigned long long*)&a.stats[ST_KEY0_PRESENT], 1ull);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 8; i++)
            if (!((livem >> i) & 1u)) bk[i] = kNoKey;
        // the chunk's buckets for the record stage (one 16-byte store)
        {
            v4u pk;
            pk.x = bk[0] | (bk[1] << 16);
            pk.y = bk[2] | (bk[3] << 16);
            pk.z = bk[4] | (bk[5] << 16);
            pk.w = bk[6] | (bk[7] << 16);
            *(v4u*)(wbk + 8 * lane) = pk;
        }
        // 4. run starts / ends; neighbouring chunks from the neighbouring lanes
        u32 prev = (u32)__shfl_up((int)bk[7], 1);
        u32 nxt = (u32)__shfl_down((int)bk[0], 1);
        if (first_chunk) prev = kNoKey;
        if (last_chunk) nxt = kNoKey;
        u32 smask = 0, emask = 0;
        {
            u32 pv = prev;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const u32 v = bk[i];
                const u32 nx = i < 7 ? bk[i + 1] : nxt;
                if (v != kNoKey) {
                    smask |= (v != pv ? 1u : 0u) << i;
                    emask |= (v != nx ? 1u : 0u) << i;
                }
                pv = v;
            }
        }
        const u32 open = (bk[0] != kNoKey && bk[0] == prev) ? 1u : 0u;  // a run continues into this chunk
        u32 T;
        const u32 ex = f2_scan16((u32)__popc(smask), &T);
        {
            // set bits only (a lane holds one or two starts and ends)
            u32 sp = ex, ep = ex - open;
            for (u32 mm = smask; mm; mm &= mm - 1u) sa[sp++] = (unsigned short)(q0 + (u32)__builtin_ctz(mm));
            for (u32 mm = emask; mm; mm &= mm - 1u) ea[ep++] = (unsigned short)(q0 + (u32)__builtin_ctz(mm));
        }
        wave_sync();
        if (a.skip & 2) continue;
        // 5. runs -> pieces of <= nmax windows -> records at consecutive
        // positions of the wave's pool chunk (one global atomic per chunk)
        for (u32 i0 = 0; i0 < T; i0 += 64) {
            const u32 i = i0 + (u32)lane;
            u32 qs = 0, n = 0;
            if (i < T) {
                qs = sa[i];
                n = (u32)ea[i] - qs + 1u;
            }
            const u32 pieces = n <= NMAX ? (n ? 1u : 0u) : (n + NMAX - 1u) / NMAX;
            u32 ptot, pb;
            if (__ballot(pieces > 15u) == 0ull) {
                pb = f2_scan16(pieces, &ptot);
            } else {
                const u32 inc = wave_incl_scan(pieces);
                pb = inc - pieces;
                ptot = (u32)__builtin_amdgcn_readlane((int)inc, 63);
            }
            const u64 room = cend - ccur;
            const u64 oc = ccur;
            u64 nbase = 0;
            if ((u64)ptot > room) {
                u64 nb = 0;
                if (lane == 0) nb = atomicAdd((unsigned long long*)a.pool_cursor, (unsigned long long)a.chunk);
                nb = readlane64(nb, 0);
                nbase = nb;
                ccur = nb + ((u64)ptot - room);
                cend = nb + a.chunk;
            } else {
                ccur += ptot;
            }
            if (n == 0) continue;
            const int r = (int)div_nw.div(qs);
            const int ps0 = (int)qs - r * nw;
            const u64 bkt = wbk[r * 8 * nchr + ps0];
            const u32* crw = codes + r * NG;
            u32 g = pb;
            for (u32 off = 0; off < n; off += NMAX, g++) {
                const u32 nn = min(NMAX, n - off);
                const int ps = ps0 + (int)off;
                u64 rec[RW];
                {
                    // words g .. g + 2 RW of the row hold bases ps .. ps + 32 RW - 8 + 31
                    const int g = ps >> 4, o = ps & 15;
                    u32 cw[2 * RW + 1];
#pragma unroll
                    for (int x = 0; x < 2 * RW + 1; x++) cw[x] = crw[g + x];
                    u32 sw[2 * RW];  // the row shifted to base ps
#pragma unroll
                    for (int x = 0; x < 2 * RW; x++) sw[x] = o ? __builtin_amdgcn_alignbit(cw[x], cw[x + 1], 32 - 2 * o) : cw[x];
                    // word 0: bucket, then bases ps ..; word j >= 1: bases ps + 32 j - 8 ..
                    rec[0] = (bkt << 48) | ((((u64)sw[0] << 32) | sw[1]) >> 16);
#pragma unroll
                    for (int j = 1; j < RW; j++)
                        rec[j] = ((((u64)sw[2 * j - 1] << 32) | sw[2 * j]) << 16) | (sw[2 * j + 1] >> 16);
                }
                const int vb = 16 + 2 * (C::KP + (int)nn - 1);
#pragma unroll
                for (int j = 0; j < RW; j++) {
                    const int bits = vb - 64 * j;
                    const u64 msk = bits >= 64 ? ~0ull : (bits <= 0 ? 0ull : (~0ull << (64 - bits)));
                    rec[j] &= msk;
                }
                rec[RW - 1] |= (u64)nn;
                const u64 dst = (u64)g < room ? oc + g : nbase + ((u64)g - room);
                if (dst < a.pool_cap && !(a.skip & 1)) {
#pragma unroll
                    for (int j = 0; j < RW; j++) a.pool[(u64)j * a.pool_cap + dst] = rec[j];
                    if (a.dig1) a.dig1[dst] = (unsigned char)bkt;
                }
            }
        }
        wave_sync();
    }
    // pad the rest of the wave's chunk with n = 0 records in bucket kNoKey
    for (u64 i = ccur + (u64)lane; i < cend; i += 64)
        if (i < a.pool_cap) {
#pragma unroll
            for (int j = 0; j < RW; j++) a.pool[(u64)j * a.pool_cap + i] = j == 0 ? ((u64)kNoKey << 48) : 0ull;
            if (a.dig1) a.dig1[i] = (unsigned char)kNoKey;
        }
    wave_add(&a.stats[ST_VALID], my_valid);
    if (__ballot(my_hole) && lane == 0) atomicOr((unsigned long long*)&a.stats[ST_KEY0_PRESENT], 1ull);
}

// ---------------------------------------------------------------------------
// F3: skm_front3_k<K> (W = 1, m = 11, 19 <= k <= 32). One lane per read: a
// wave takes 64 reads (a tile) and all lanes walk their reads' m-mer
// positions in lock-step, so a position, its window and every shift are
// wave-uniform and the per-window work is a handful of VALU operations with
// no cross-lane traffic:
//   - positions come in blocks of B (16 for k - 10 >= 17, else 8) inside a
//     code word pair: the B m-mer hashes, their prefix minima (one running
//     register) and suffix minima (kept for the next two blocks)
//   - a window of k - 10 m-mers ends in block b and starts in block b - 1 or
//     b - 2 (B < k - 10 < 2B), so its minimum is min(suffix, prefix) or
//     min3(suffix, whole block b - 1, prefix) (van Herk / Gil-Werman)
//   - a lane whose bucket changes pushes the run that ended (start, end,
//     bucket, read) to the wave's descriptor ring (ballot + mbcnt)
//   - every 64 descriptors become records: one descriptor per lane, pieces of
//     <= nmax windows, record words from the read's row of code words in LDS,
//     consecutive lanes at consecutive pool slots (coalesced stores)
// Reads with not-ACGT bases or aligned all-A halves (possible key 0) make the
// tile take the per-window liveness checks of F2's slow path.
// Same records as F2 (same runs, same pieces) up to their order in the pool.
// ---------------------------------------------------------------------------
template <int V>
struct F3Tag {
    static constexpr int value = V;
};

// f(F3Tag<I>{}) for I in [I0, N), unrolled by construction
template <int I0, int N, typename F>
__device__ __forceinline__ void f3_static_for(F&& f) {
    if constexpr (I0 < N) {
        f(F3Tag<I0>{});
        f3_static_for<I0 + 1, N>(f);
    }
}

template <int K>
struct F3Cfg {
    static constexpr int WM = K - 10;            // m-mers per window (m = 11)
    static constexpr int B = WM >= 17 ? 16 : 8;  // positions per block
    static constexpr int E = WM - 1;             // window span - 1
    static constexpr int D = E - B;              // a block's windows that start two blocks back
    static_assert(D >= 0 && D < B, "block geometry: B < k - 10 <= 2B");
};

#ifndef KC_F3_WPE
#define KC_F3_WPE 4  // F3: waves per SIMD the register budget is sized for
#endif
// per wave (u64): < 64 + 2 x 64 descriptors between drain checks, then a
// spare slot per lane (with a check every 4 windows and 384 slots, a
// wave's LDS at L = 150 kept F3 to 3 waves per SIMD instead of 4)
constexpr int kF3Ring = 256;
constexpr int kF3Check = 2;  // windows between drain checks

struct F3Args {
    const u32* codes;             // kernel E output, G u32 per read
    const unsigned short* inval;  //   not-ACGT masks, G u16 per read
    u64 n_reads, ntiles;
    int G, nw, np, NG;  // np = L - 10 m-mer positions; NG: LDS row stride (words, odd)
    u32 wbytes;         // a wave's LDS: ring, read flags, 64 rows
    u64 chunk;
    u64* pool;
    u64 pool_cap;
    u64* pool_cursor;
    unsigned char* dig1;
    u64* stats;
    int skip;  // timing experiments only (KC_F_SKIP): 1 record stores, 2 runs + records
    // KC_FLAG_VARLEN: read r's own length (slot positions past it are
    // not-ACGT padding in inval); nullptr: every read has L bases
    const unsigned short* rlen;
};

// 22-bit m-mer at base I of the 32 bases {c0, c1} (I constant after unrolling)
__device__ __forceinline__ u32 f3_mmer(u32 c0, u32 c1, int I) {
    return (I <= 5 ? (c0 >> (10 - 2 * I)) : __builtin_amdgcn_alignbit(c0, c1, 42 - 2 * I)) & 0x3fffffu;
}

// 64 not-ACGT bits from base b of a read (MSB = base b; bases < 0 none)
__device__ __forceinline__ u64 f3_inv64(const unsigned short* __restrict__ iv, int G, int b) {
    const int b0 = b < 0 ? 0 : b;
    const int g = b0 >> 4, sh = b0 & 15;
    u32 w[5];
#pragma unroll
    for (int t = 0; t < 5; t++) w[t] = g + t < G ? (u32)iv[g + t] : 0u;
    u64 x = ((u64)w[0] << 48) | ((u64)w[1] << 32) | ((u64)w[2] << 16) | (u64)w[3];
    if (sh) x = (x << sh) | ((u64)w[4] >> (16 - sh));
    return b < 0 ? x >> (-b) : x;
}

template <int K>
__global__ __launch_bounds__(kSkmBlock) __attribute__((amdgpu_waves_per_eu(KC_F3_WPE, 8))) void skm_front3_k(F3Args a) {
    using C = F3Cfg<K>;
    using C2 = F2Cfg<1, K>;
    constexpr int B = C::B, E = C::E, D = C::D;
    constexpr int RW = 2;
    constexpr u32 NMAX = (u32)C2::NMAX;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    unsigned char* wb = smem + (size_t)wave * a.wbytes;
    u64* ring = (u64*)wb;
    u64* const spare = ring + (kF3Ring - 64 + lane_id());  // the lane's slot when it pushes nothing
    u32* rflag = (u32*)(wb + kF3Ring * 8);
    u32* codes = rflag + 64;                 // 64 rows x NG words
    u32* stage = codes + 64 * a.NG;          // next tile: 64 G code words, then 32 G mask dwords (u16 pairs)
    const int G = a.G, NG = a.NG, nw = a.nw, np = a.np;
    const int L = np + 10;
    const u64 wid = (u64)blockIdx.x * (kSkmBlock / 64) + wave;
    const u64 nwaves = (u64)gridDim.x * (kSkmBlock / 64);
    for (int i = lane; i < 64 * NG; i += 64) codes[i] = 0;
    const FastDivU div_g((u32)G);
    const u32* crow = codes + lane * NG;
    const u32 ltag = (u32)lane << 16;
    u64 my_valid = 0, my_zero = 0;
    bool my_hole = false;
    u64 ccur = 0, cend = 0;  // the wave's pool chunk (wave-uniform)
    u32 qn = 0;              // descriptors in the ring (wave-uniform)
    // records of the first cnt descriptors (one per lane); the rest move down
    auto drain = [&](u32 cnt) {
        wave_sync();
        const bool has = (u32)lane < cnt;
        const u64 d = has ? ring[lane] : 0ull;
        for (u32 i = cnt + (u32)lane; i < qn; i += 64) ring[i - cnt] = ring[i];
        qn -= cnt;
        if (a.skip & 8) return;  // timing experiments: descriptors only
        const u32 lo = (u32)d, hi = (u32)(d >> 32);
        const u32 s0 = lo >> 16;
        const u64 bkt = lo & 0xffffu;
        const u32 n = has ? (hi & 0xffffu) - s0 + 1u : 0u;
        // pool slots: one piece per run unless a run is longer than nmax
        u32 ptot, pb;
        const bool multi = __builtin_amdgcn_ballot_w64(n > NMAX) != 0ull;
        u32 pieces = has ? 1u : 0u;
        if (!multi) {
            pb = (u32)lane;  // the descriptors sit in lanes 0 .. cnt - 1
            ptot = cnt;
        } else {
            pieces = (n + NMAX - 1u) / NMAX;
            const u32 inc = wave_incl_scan(pieces);
            pb = inc - pieces;
            ptot = (u32)__builtin_amdgcn_readlane((int)inc, 63);
        }
        const u64 room = cend - ccur;
        u64 b0 = ccur, b1 = 0;  // slot g: b0 + g below room, else b1 + g
        if ((u64)ptot > room) {
            u64 nb = 0;
            if (lane == 0) nb = atomicAdd((unsigned long long*)a.pool_cursor, (unsigned long long)a.chunk);
            nb = readlane64(nb, 0);
            b1 = nb - room;
            ccur = nb + ((u64)ptot - room);
            cend = nb + a.chunk;
        } else {
            ccur += ptot;
        }
        const u32* crw = codes + (hi >> 16) * NG;
        // record of the piece of nn windows from window ps
        auto piece = [&](int ps, u32 nn, u64 (&rec)[RW]) {
            const int g = ps >> 4, o = ps & 15;
            u32 cw[2 * RW + 1];
#pragma unroll
            for (int x = 0; x < 2 * RW + 1; x++) cw[x] = crw[g + x];
            u32 sw[2 * RW];
#pragma unroll
            for (int x = 0; x < 2 * RW; x++) sw[x] = o ? __builtin_amdgcn_alignbit(cw[x], cw[x + 1], 32 - 2 * o) : cw[x];
            rec[0] = (bkt << 48) | ((((u64)sw[0] << 32) | sw[1]) >> 16);
#pragma unroll
            for (int j = 1; j < RW; j++) rec[j] = ((((u64)sw[2 * j - 1] << 32) | sw[2 * j]) << 16) | (sw[2 * j + 1] >> 16);
            // keep the 16 + 2 (K' + nn - 1) bits of the record
            const int vb = 16 + 2 * (C2::KP + (int)nn - 1);
#pragma unroll
            for (int j = 0; j < RW; j++) {
                const int bits = vb - 64 * j;
                if (bits < 64) rec[j] &= bits <= 0 ? 0ull : (~0ull << (64 - bits));
            }
            rec[RW - 1] |= (u64)nn;
        };
        // the usual drain (wave-uniform test): one piece per lane, all in the
        // current chunk and the pool, slot b0 + lane (uniform bases, 32-bit
        // lane offsets, no 64-bit slot arithmetic per lane)
        if (!multi && (u64)ptot <= room && b0 + (u64)ptot <= a.pool_cap && !(a.skip & 1)) {
            if (has) {
                u64 rec[RW];
                piece((int)s0, min(NMAX, n), rec);  // n <= NMAX here (!multi)
                u64* const w0 = a.pool + readlane64(b0, 0);
#pragma unroll
                for (int j = 0; j < RW; j++) (w0 + (u64)j * a.pool_cap)[(u32)lane] = rec[j];
                if (a.dig1) (a.dig1 + readlane64(b0, 0))[(u32)lane] = (unsigned char)bkt;
            }
            return;
        }
        for (u32 p = 0; p < pieces; p++) {
            const u32 off = p * NMAX;
            u64 rec[RW];
            piece((int)(s0 + off), min(NMAX, n - off), rec);
            const u32 gq = pb + p;
            const u64 dst = ((u64)gq < room ? b0 : b1) + gq;
            if (dst < a.pool_cap && !(a.skip & 1)) {
#pragma unroll
                for (int j = 0; j < RW; j++) a.pool[(u64)j * a.pool_cap + dst] = rec[j];
                if (a.dig1) a.dig1[dst] = (unsigned char)bkt;
            }
        }
    };
    // a run ended at window w - 1 in the lanes of `ended` (prev: its bucket,
    // s: its first window); descriptor = read lane | last window, first
    // window | bucket
    auto push = [&](bool ended, u64 pm, int wlast, u32 s, u32 prev) {
        if (ended) {
            const u32 rank = __builtin_amdgcn_mbcnt_hi((u32)(pm >> 32), __builtin_amdgcn_mbcnt_lo((u32)pm, 0u));
            ring[qn + rank] = ((u64)(ltag | (u32)wlast) << 32) | ((s << 16) | prev);
        }
        qn += (u32)__popcll(pm);
    };
    // a tile's code words and masks into the staging area by LDS DMA (no
    // registers held while in flight); lanes past the tile load its first word
    const int ngw = 64 * G, nmw = 32 * G;  // staged dwords: codes, masks
    auto prefetch = [&](u64 t) {
        if (t >= a.ntiles) return;
        const int nwords = (int)min((u64)64, a.n_reads - t * 64) * G;
        const u32* cg = a.codes + t * 64 * (u64)G;
        for (int j = 0; j < ngw; j += 64) {
            const int it = j + lane < nwords ? j + lane : 0;
            __builtin_amdgcn_global_load_lds((const void*)(cg + it), (__attribute__((address_space(3))) void*)(stage + j), 4, 0, 0);
        }
        const u32* mg = (const u32*)(a.inval + t * 64 * (u64)G);  // 4-byte aligned (launch checks a.inval)
        for (int j = 0; j < nmw; j += 64) {
            const int it = 2 * (j + lane) < nwords ? j + lane : 0;
            __builtin_amdgcn_global_load_lds((const void*)(mg + it), (__attribute__((address_space(3))) void*)(stage + ngw + j), 4, 0, 0);
        }
    };
    prefetch(wid);
    wave_sync();
    for (u64 tile = wid; tile < a.ntiles; tile += nwaves) {
        const u64 r0 = tile * 64;
        const int nr = (int)min((u64)64, a.n_reads - r0);
        // the lane's read length (variable-length reads, one-pass rows), loaded
        // before the wait below: a global load issued after the next tile's
        // prefetch would wait for the whole prefetch (in-order vmcnt)
        const int my_rl = (a.rlen && lane < nr) ? (int)a.rlen[r0 + (u64)lane] : L;
        // 1. the tile's staged code words into the rows; read flags (not-ACGT
        // bases, aligned all-A halves inside the read)
        rflag[lane] = 0;
        int* rls = (int*)ring;  // the lengths by row (the ring is empty between tiles)
        rls[lane] = my_rl;
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the staging DMA has landed
        wave_sync();
        {
            const int nwords = nr * G;
            for (int it = lane; it < nwords; it += 64) {
                const u32 cw = stage[it];
                const u32 iv = (stage[ngw + (it >> 1)] >> (16 * (it & 1))) & 0xffffu;
                const int r = (int)div_g.div((u32)it), g = it - r * G;
                codes[r * NG + g] = cw;
                int lr = L;  // the read's own length
                u32 ivr = iv;
                if (a.rlen) {
                    // a variable-length read: the padding past its end is no
                    // bad base (its windows end with the read, below)
                    lr = rls[r];
                    const int o = lr - 16 * g;
                    ivr = o >= 16 ? iv : (o <= 0 ? 0u : iv & ~((1u << (16 - o)) - 1u));
                }
                const bool za = ((cw >> 16) == 0u && 16 * g + 8 <= lr) || ((cw & 0xffffu) == 0u && 16 * g + 16 <= lr);
                const u32 f = (ivr ? 1u : 0u) | (za ? 2u : 0u);
                if (f) atomicOr(&rflag[r], f);
            }
        }
        wave_sync();
        prefetch(tile + nwaves);
        const u32 fl = lane < nr ? rflag[lane] : 0u;
        const int slow = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_ballot_w64(fl != 0u) != 0ull ? 1 : 0);  // uniform
        const unsigned short* ivg = a.inval + (r0 + (u64)(lane < nr ? lane : 0)) * (u64)G;
        // 2. lock-step walk over the positions
        u32 Sp[B];                 // suffix minima of the previous block
        u32 St[D > 0 ? D : 1];     // ... of the block before it, last D
        u32 prev = kNoKey, s = 0;  // the open run: bucket, first window
#pragma unroll
        for (int i = 0; i < B; i++) Sp[i] = ~0u;
#pragma unroll
        for (int i = 0; i < (D > 0 ? D : 1); i++) St[i] = ~0u;
        const bool fast = !slow && !(a.skip & 2);
        // windows of the lane's read (variable-length reads: its own; windows
        // from nwr on are not windows, their bucket is kNoKey); vt: a read of
        // the tile is shorter than the slot (wave-uniform). A row of length 0
        // (one-pass index: a chunk's rows past its records) is no read: it
        // pushes nothing (live) and does not make the interior blocks take
        // the per-window length test (vtf)
        int nwr = nw;
        if (a.rlen && lane < nr) nwr = max(0, my_rl - K + 1);
        const bool live = lane < nr && my_rl != 0;
        const u64 livem = __builtin_amdgcn_ballot_w64(live);
        const bool vt = a.rlen != nullptr && __builtin_amdgcn_ballot_w64(lane < nr && nwr < nw) != 0ull;
        const bool vtf = a.rlen != nullptr && __builtin_amdgcn_ballot_w64(live && nwr < nw) != 0ull;
        const int g_lo = (E + 1 + 15) / 16;                  // first block whose windows are all >= 1
        const int g_hi = np >= 16 ? (np - 16) / 16 + 1 : 0;  // blocks ending before np
        u32 c0 = crow[0];
        for (int g = 0; 16 * g < ((a.skip & 4) ? 0 : np); g++) {
            const u32 c1 = crow[g + 1];
            // interior block of a tile without flagged reads: every window
            // exists (w >= 1) and is live, no per-window branch; lanes without a
            // run to push write their spare ring slot
            auto fast_block = [&](auto tag, auto vtag) {
                constexpr int OFF = decltype(tag)::value;
                constexpr bool VT = decltype(vtag)::value;
                const int p0 = 16 * g + OFF;
                u32 h[B];
#pragma unroll
                for (int i = 0; i < B; i++) h[i] = mul_u24(f3_mmer(c0, c1, OFF + i) ^ 0xd1e995u, 0x9e3779u);
                u32 P = h[0];
                const u32 wv0 = (u32)(p0 - E);  // window of j = 0
                // the open run as one register, first window << 16 | bucket:
                // a boundary replaces it, its low half is prev (16-bit compare)
                u32 sl = (s << 16) | prev;
                f3_static_for<0, B>([&](auto jt) {
                    constexpr int j = decltype(jt)::value;
                    if constexpr (j > 0) P = min(P, h[j]);
                    u32 v;
                    if constexpr (j < D)
                        v = min(min(St[j], Sp[0]), P);
                    else
                        v = min(Sp[j - D], P);
                    u32 u = min(v & 0xffffu, kNoKey - 1u);
                    const u32 w = wv0 + (u32)j;
                    if constexpr (VT) u = (int)w < nwr ? u : kNoKey;
                    const bool bnd = (unsigned short)u != (unsigned short)sl;
                    const u64 pm = __builtin_amdgcn_ballot_w64(bnd) & livem;
                    u32 mb = __builtin_amdgcn_mbcnt_hi((u32)(pm >> 32), __builtin_amdgcn_mbcnt_lo((u32)pm, 0u));
                    // the rank in every lane, then a select: without this the
                    // compiler sinks the rank into a branch on bnd and the
                    // select into a second one (~8 more SALU per window)
                    asm volatile("" : "+v"(mb));
                    // every lane stores (a lane that pushes nothing to its spare
                    // slot): faster than a store by the pushing lanes only,
                    // whose exec mask costs more than the bank conflicts it
                    // avoids (7.91-7.97 vs 7.85-7.88 ms at cfg2)
                    u64* const slot = (bnd && live) ? ring + qn + mb : spare;
                    *slot = ((u64)(ltag | (w - 1u)) << 32) | sl;
                    qn += (u32)__popcll(pm);
                    u32 wsh = w << 16;
                    asm volatile("" : "+s"(wsh));  // one SGPR, not (first << 16) | u | (j << 16)
                    sl = bnd ? (wsh | u) : sl;
                    if constexpr (j % kF3Check == kF3Check - 1)
                        while (qn >= 64u) drain(64u);
                });
                s = sl >> 16;
                prev = sl & 0xffffu;
#pragma unroll
                for (int x = 0; x < D; x++) St[x] = Sp[B - D + x];
                Sp[B - 1] = h[B - 1];
#pragma unroll
                for (int i = B - 2; i >= 0; i--) Sp[i] = min(h[i], Sp[i + 1]);
            };
            auto block = [&](auto tag) {
                constexpr int OFF = decltype(tag)::value;
                const int p0 = 16 * g + OFF;
                if (p0 >= np) return;
                u32 h[B];
#pragma unroll
                for (int i = 0; i < B; i++) h[i] = mul_u24(f3_mmer(c0, c1, OFF + i) ^ 0xd1e995u, 0x9e3779u);
                u32 deadm = 0;
                if (slow && (fl & 1u)) {
                    const u64 X = f3_inv64(ivg, G, p0 - E);
                    constexpr u64 KM = ~0ull << (64 - K);  // a window's K bases
#pragma unroll
                    for (int j = 0; j < B; j++) deadm |= ((X & (KM >> j)) ? 1u : 0u) << j;
                }
                u32 P = h[0];
                f3_static_for<0, B>([&](auto jt) {
                    constexpr int j = decltype(jt)::value;
                    if constexpr (j > 0) P = min(P, h[j]);
                    const int w = p0 + j - E;
                    if (w >= 0 && w < nw) {  // wave-uniform
                        u32 v;
                        if constexpr (j < D)
                            v = min(min(St[j], Sp[0]), P);
                        else
                            v = min(Sp[j - D], P);
                        u32 u = min(v & 0xffffu, kNoKey - 1u);
                        const bool beyond = vt && w >= nwr;  // past a variable-length read's windows
                        if (slow) {
                            const bool dead = (deadm >> j) & 1u;
                            bool zero = false;
                            if ((fl & 2u) && !dead && !beyond) zero = (f2_code_word(crow, w) & C2::LAST_MASK) == 0ull;
                            if (lane < nr) {
                                my_valid += (dead || beyond) ? 0u : 1u;
                                my_zero += zero ? 1u : 0u;
                                my_hole |= dead && !beyond;
                            }
                            if (dead || zero) u = kNoKey;
                        }
                        if (beyond) u = kNoKey;
                        if (w == 0) {
                            s = 0;
                        } else if (!(a.skip & 2)) {
                            if (!slow) {
                                const bool bnd = u != prev;
                                push(bnd && live, __builtin_amdgcn_ballot_w64(bnd) & livem, w - 1, s, prev);
                                if (bnd) s = (u32)w;
                            } else {
                                const bool ended = u != prev && live && prev != kNoKey;
                                const u64 pm = __builtin_amdgcn_ballot_w64(ended);
                                push(ended, pm, w - 1, s, prev);
                                if (u != prev) s = (u32)w;
                            }
                        }
                        prev = u;
                    }
                    if constexpr (j % kF3Check == kF3Check - 1)
                        while (qn >= 64u) drain(64u);
                });
#pragma unroll
                for (int x = 0; x < D; x++) St[x] = Sp[B - D + x];
                Sp[B - 1] = h[B - 1];
#pragma unroll
                for (int i = B - 2; i >= 0; i--) Sp[i] = min(h[i], Sp[i + 1]);
            };
            if (fast && g >= g_lo && g < g_hi) {
                if (vtf) {
                    fast_block(F3Tag<0>{}, std::true_type{});
                    if constexpr (B == 8) fast_block(F3Tag<8>{}, std::true_type{});
                } else {
                    fast_block(F3Tag<0>{}, std::false_type{});
                    if constexpr (B == 8) fast_block(F3Tag<8>{}, std::false_type{});
                }
            } else {
                block(F3Tag<0>{});
                if constexpr (B == 8) block(F3Tag<8>{});
            }
            c0 = c1;
        }
        // the open runs end at the last window
        {
            const bool ended = prev != kNoKey && live && !(a.skip & 2);
            push(ended, __builtin_amdgcn_ballot_w64(ended), nw - 1, s, prev);
        }
        while (qn) drain(min(64u, qn));
        if (!slow && lane < nr) my_valid += (u64)nwr;
        wave_sync();
    }
    // pad the rest of the wave's chunk with n = 0 records in bucket kNoKey
    for (u64 i = ccur + (u64)lane; i < cend; i += 64)
        if (i < a.pool_cap) {
#pragma unroll
            for (int j = 0; j < RW; j++) a.pool[(u64)j * a.pool_cap + i] = j == 0 ? ((u64)kNoKey << 48) : 0ull;
            if (a.dig1) a.dig1[i] = (unsigned char)kNoKey;
        }
    wave_add(&a.stats[ST_VALID], my_valid);
    const u64 zsum = my_zero;
    if (__builtin_amdgcn_ballot_w64(zsum != 0ull)) {
        wave_add(&a.stats[ST_KEY0], zsum);
        if (lane == 0) atomicOr((unsigned long long*)&a.stats[ST_KEY0_PRESENT], 1ull);
    }
    if (__builtin_amdgcn_ballot_w64(my_hole) && lane == 0) atomicOr((unsigned long long*)&a.stats[ST_KEY0_PRESENT], 1ull);
}

// F3 geometry: false when F3 does not apply
static bool f3_args(const CountLaunch& l, const SkmGeom& g, F3Args* a, size_t* lds) {
    const int W = (l.k + 31) / 32;
    if (W != 1 || g.m != 11 || l.k < 19 || l.k > 32 || test_hook("KC_NO_F3")) return false;
    if (((uintptr_t)l.inval & 3) || ((uintptr_t)l.codes & 3)) return false;  // dword DMA of the masks
    const int nw = l.L - l.k + 1;
    if (nw <= 0 || nw > 65535) return false;
    a->G = groups_per_read(l.L);
    a->nw = nw;
    a->np = l.L - 10;
    // rows: hash pairs read words g, g + 1 (g <= (np - 1) / 16), records
    // words (ps >> 4) .. + 2 RW (ps < nw), zero tests + 2
    int ng = a->G + 1;
    if (ng < (nw - 1) / 16 + 5) ng = (nw - 1) / 16 + 5;
    ng |= 1;  // odd stride: a lane per row, no bank conflicts
    a->NG = ng;
    // ring, read flags, rows, staging (codes + masks of the next tile)
    const size_t wbytes = (size_t)kF3Ring * 8 + 64 * 4 + (size_t)64 * ng * 4 + (size_t)96 * a->G * 4;
    if (wbytes > 40 * 1024) return false;
    a->wbytes = (u32)wbytes;
    *lds = (size_t)(kSkmBlock / 64) * wbytes;
    return true;
}

// Whether F3 counts (L, k) batches (its geometry and LDS budget; the codes'
// alignment is the batch split's, kept even by count_reads_skm): the one-pass
// FASTQ index is used only then, since only F3 skips its empty rows for free
bool skm_f3_applies(int L, int k) {
    const SkmGeom g = skm_geometry(L, k);
    if (!g.ok) return false;
    static const uint32_t aligned[4] = {0, 0, 0, 0};
    CountLaunch l{};
    l.L = L;
    l.k = k;
    l.codes = aligned;
    l.inval = (const uint16_t*)aligned;
    F3Args a;
    size_t lds = 0;
    return f3_args(l, g, &a, &lds);
}

// F2 geometry for (L, k) (W = 1, m = 11): false when F2 does not apply
static bool f2_args(const CountLaunch& l, const SkmGeom& g, F2Args* a, size_t* lds) {
    const int W = (l.k + 31) / 32;
    if (W != 1 || g.m != 11 || l.k < 18 || l.k > 32 || test_hook("KC_NO_F2")) return false;
    const int nw = l.L - l.k + 1;
    const int nchr = (nw + 7) / 8;
    if (nchr > 64 || nw <= 0) return false;
    const int RW = W + 1;
    a->G = groups_per_read(l.L);
    a->nw = nw;
    a->nchr = nchr;
    a->R = 64 / nchr;
    // hash positions needed: [0, 8 nchr + wm + 7)
    const int wm = l.k - 11 + 1;
    a->NI = (8 * nchr + wm + 7 + 15) / 16;
    a->HSK = 18 * a->NI + 1;
    // code words: records read 3 words from (ps + 32 j - 8) / 16, hashes NI + 1
    int ng = (8 * nchr + 32 * RW) / 16 + 2 * RW + 3;
    if (ng < a->NI + 2) ng = a->NI + 2;
    if (ng < a->G + 1) ng = a->G + 1;
    a->NG = ng;
    size_t p = (size_t)a->R * ng * 4;
    a->o_inval = (u32)p;
    p += (size_t)a->R * ng * 4;
    a->o_hm = (u32)p;
    p += (size_t)a->R * a->HSK * 4;
    a->o_rflag = (u32)p;
    p += 64 * 4;
    a->o_sa = (u32)p;
    p += (size_t)a->R * nchr * 8 * 2;
    a->o_ea = (u32)p;
    p += (size_t)a->R * nchr * 8 * 2;
    p = (p + 15) & ~(size_t)15;
    a->o_bk = (u32)p;
    p += 64 * 8 * 2;
    a->wbytes = (u32)p;
    *lds = p * (kSkmBlock / 64);
    if (*lds > 64 * 1024) return false;
    if ((u64)a->NI * 64 >= 65536 || (u64)a->G * 64 * kF2Pf >= 65536) return false;  // FastDivU range
    return true;
}

SkmGeom skm_geometry(int L, int k) {
    SkmGeom g;
    g.ok = false;
    const int W = (k + 31) / 32;
    const int RW = W + 1;
    if (W > 3 || k < 18 || L < k) return g;
    const bool mask_last = ((k + 3) / 4) < 8 * W;
    g.Kp = mask_last ? k : 32 * W;
    g.nmax = 32 * RW - 10 - g.Kp;
    if (g.nmax > 63) g.nmax = 63;
    // m-mers: a window's minimizer lives ~(k - m + 1) windows; runs longer
    // than nmax are split, so aim k - m + 1 <= nmax (m in [11, 24])
    int m = k - g.nmax + 1;
    int mmin = 11;
    if (const int e = experiment_knob("KC_SKM_MMIN")) mmin = e;
    if (m < mmin) m = mmin;
    if (m > 24) m = 24;
    if (k - m + 1 < 8) m = k - 7;
    g.m = m;
    const int nw = L - k + 1;
    const int nchr = (nw + 7) / 8;
    if (nw > 4096) return g;  // a tile's records must fit one pool chunk
    g.NG = (L + 32 * RW + 64) / 16 + 3;
    g.HS = L - m + 8;
    // a wave tile: R reads whose 8-window chunks fill the wave's 64 lanes
    int R = 64 / nchr;
    if (R < 1) R = 1;
    g.R = R;
    int ipr = 64 / R;  // hash items per read
    if (ipr < 1) ipr = 1;
    g.hq = (g.HS + ipr - 1) / ipr;
    if (g.hq > 32 - m + 1) g.hq = 32 - m + 1;
    if (g.hq > 22) g.hq = 22;
    if (g.hq < 1) g.hq = 1;
    g.lds = (size_t)(kSkmBlock / 64) * skm_lds_layout(R, g.NG, (g.HS + g.hq - 1) / g.hq * g.hq, nw).total;
    if (g.lds > 160 * 1024) return g;
    g.ok = true;
    return g;
}

hipError_t launch_skm_front(const CountLaunch& l, const SkmGeom& g, uint64_t* pool, uint64_t pool_cap,
                            uint64_t* pool_cursor, int grid_cap, hipStream_t s, uint8_t* dig1) {
    if (l.n_reads == 0) return hipSuccess;
    if (!g.ok || !l.codes || !l.inval) return hipErrorInvalidValue;
    SkmArgs a;
    a.codes = l.codes;
    a.inval = (const unsigned short*)l.inval;
    a.G = groups_per_read(l.L);
    a.n_reads = l.n_reads;
    a.L = l.L;
    a.k = l.k;
    a.m = g.m;
    a.Kp = g.Kp;
    a.nmax = g.nmax;
    a.R = g.R;
    a.NG = g.NG;
    a.HS = g.HS;
    a.pool = pool;
    a.pool_cap = pool_cap;
    a.pool_cursor = pool_cursor;
    a.dig1 = dig1;
    a.stats = l.stats;
    a.hq = g.hq;
    a.chunk = (u64)g.R * (u64)(l.L - l.k + 1);
    if (a.chunk < 1024) a.chunk = 1024;
    a.skip = experiment_knob("KC_F_SKIP");
    {
        F3Args f3;
        size_t f3lds = 0;
        if (f3_args(l, g, &f3, &f3lds)) {
            f3.codes = l.codes;
            f3.inval = (const unsigned short*)l.inval;
            f3.n_reads = l.n_reads;
            f3.ntiles = (l.n_reads + 63) / 64;
            // a drain's pieces: 64 runs of <= nw windows, nmax per piece
            f3.chunk = 64 * (u64)((f3.nw + g.nmax - 1) / g.nmax);
            if (f3.chunk < 1024) f3.chunk = 1024;
            f3.pool = pool;
            f3.pool_cap = pool_cap;
            f3.pool_cursor = pool_cursor;
            f3.dig1 = dig1;
            f3.stats = l.stats;
            f3.rlen = (const unsigned short*)l.rlen;
            f3.skip = experiment_knob("KC_F_SKIP");
            int per_cu = 0, n_cu = 0, dev = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
            const u64 nwg = (f3.ntiles + kSkmBlock / 64 - 1) / (kSkmBlock / 64);
#define KC_F3(KK)                                                                                               \
    case KK:                                                                                                    \
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, skm_front3_k<KK>, kSkmBlock, f3lds);       \
        {                                                                                                       \
            u64 cap = (per_cu > 0 && n_cu > 0) ? (u64)per_cu * (u64)n_cu : (u64)grid_cap;                      \
            if (cap > (u64)grid_cap) cap = (u64)grid_cap;                                                       \
            hipLaunchKernelGGL((skm_front3_k<KK>), dim3((int)hmin(nwg, cap)), dim3(kSkmBlock), f3lds, s, f3);    \
        }                                                                                                       \
        break;
            switch (l.k) {
                KC_F3(19) KC_F3(20) KC_F3(21) KC_F3(22) KC_F3(23) KC_F3(24) KC_F3(25) KC_F3(26)
                KC_F3(27) KC_F3(28) KC_F3(29) KC_F3(30) KC_F3(31) KC_F3(32)
            default: return hipErrorInvalidValue;
            }
#undef KC_F3
            return hipGetLastError();
        }
    }
    {
        F2Args f2;
        size_t f2lds = 0;
        if (f2_args(l, g, &f2, &f2lds)) {
            f2.codes = l.codes;
            f2.inval = (const unsigned short*)l.inval;
            f2.n_reads = l.n_reads;
            f2.ntiles = (l.n_reads + f2.R - 1) / f2.R;
            f2.chunk = (u64)f2.R * (u64)f2.nw;
            if (f2.chunk < 1024) f2.chunk = 1024;
            f2.pool = pool;
            f2.pool_cap = pool_cap;
            f2.pool_cursor = pool_cursor;
            f2.dig1 = dig1;
            f2.stats = l.stats;
            f2.skip = experiment_knob("KC_F_SKIP");
            int per_cu = 0, n_cu = 0, dev = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
#define KC_F2(KK)                                                                                               \
    case KK:                                                                                                    \
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, skm_front2_k<1, KK>, kSkmBlock, f2lds);    \
        {                                                                                                       \
            u64 cap = (per_cu > 0 && n_cu > 0) ? (u64)per_cu * (u64)n_cu : (u64)grid_cap;                      \
            if (cap > (u64)grid_cap) cap = (u64)grid_cap;                                                       \
            hipLaunchKernelGGL((skm_front2_k<1, KK>), dim3((int)hmin(f2.ntiles, cap)), dim3(kSkmBlock), f2lds, \
                               s, f2);                                                                          \
        }                                                                                                       \
        break;
            switch (l.k) {
                KC_F2(18) KC_F2(19) KC_F2(20) KC_F2(21) KC_F2(22) KC_F2(23) KC_F2(24) KC_F2(25)
                KC_F2(26) KC_F2(27) KC_F2(28) KC_F2(29) KC_F2(30) KC_F2(31) KC_F2(32)
            default: return hipErrorInvalidValue;
            }
#undef KC_F2
            return hipGetLastError();
        }
    }
    const u64 tiles = (l.n_reads + g.R - 1) / g.R;
    const int W = (l.k + 31) / 32;
    // one wave of workgroups: every workgroup walks the same number of tiles
    int per_cu = 0, n_cu = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (W == 1) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, skm_front_k<1>, kSkmBlock, g.lds);
    else if (W == 2) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, skm_front_k<2>, kSkmBlock, g.lds);
    else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, skm_front_k<3>, kSkmBlock, g.lds);
    u64 cap = (per_cu > 0 && n_cu > 0) ? (u64)per_cu * (u64)n_cu : (u64)grid_cap;
    if (cap > (u64)grid_cap) cap = (u64)grid_cap;
    const int grid = (int)hmin(tiles, cap);
    switch (W) {
    case 1: hipLaunchKernelGGL(skm_front_k<1>, dim3(grid), dim3(kSkmBlock), g.lds, s, a); break;
    case 2: hipLaunchKernelGGL(skm_front_k<2>, dim3(grid), dim3(kSkmBlock), g.lds, s, a); break;
    case 3: hipLaunchKernelGGL(skm_front_k<3>, dim3(grid), dim3(kSkmBlock), g.lds, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// rp_*: two-level radix grouping of SoA items by the 16 bits word0 >> 48
// (generalizes P3 to any word count, an optional u32 payload, a digit taken
// from word0 at any shift, and a digit byte emitted for the next level).
// Regions: region r holds tiles [tpre[r], tpre[r+1]); tile i of r starts at
// rstart[r] + i * TILE. Level 1 is one region; level 2 takes level 1's 256
// digit regions, so its digit-major positions give (high byte, low byte)
// order. Ranks inside a tile are unstable (LDS atomics): only grouping is
// needed (records, and the keys of one group are distinct or summed later).
// ---------------------------------------------------------------------------

// radix-scatter LDS budget per workgroup (items) and workgroups per CU
#ifndef KC_RP_LDS
#define KC_RP_LDS 143808
#endif
#ifndef KC_RP_WPC
#define KC_RP_WPC 1
#endif

// threads per radix-scatter workgroup (variant builds: KC_RP_BLOCK=512 with
// KC_RP_WPC=2 and half the LDS budget runs two workgroups per CU)
#ifndef KC_RP_BLOCK
#define KC_RP_BLOCK 1024
#endif
constexpr int kRpBlock = KC_RP_BLOCK;
constexpr int kRpWaves = kRpBlock / 64;

template <int NW, bool PAY>
struct RpCfg {
    static constexpr int BYTES = 8 * NW + (PAY ? 4 : 0);
    static constexpr int K0 = KC_RP_LDS / (BYTES * kRpBlock);
    static constexpr int KPT = K0 > 16 ? 16 : K0;
    static constexpr int TILE = kRpBlock * KPT;
};

int rp_tile(int NW, bool pay) {
    const int bytes = 8 * NW + (pay ? 4 : 0);
    int kpt = KC_RP_LDS / (bytes * kRpBlock);
    if (kpt > 16) kpt = 16;
    return kRpBlock * kpt;
}

__device__ __forceinline__ void rp_tile_range(const u64* __restrict__ rstart, const u64* __restrict__ tpre, int nreg,
                                              u64 t, u64 TILE, u64* lo, u64* hi) {
    int a = 0, b = nreg;  // region r with tpre[r] <= t < tpre[r+1]
    while (b - a > 1) {
        const int mid = (a + b) >> 1;
        if (tpre[mid] <= t)
            a = mid;
        else
            b = mid;
    }
    const u64 st = rstart[a] + (t - tpre[a]) * TILE;
    *lo = st;
    *hi = min(st + TILE, rstart[a + 1]);
}

// Tile histograms (tile-major u32 counts): digit = digs[i] when digs is given,
// else (w0[i] >> shift) & 255.
__global__ __launch_bounds__(kBlock) void rp_upsweep_k(const unsigned char* __restrict__ digs,
                                                       const u64* __restrict__ w0, int shift,
                                                       const u64* __restrict__ rstart, const u64* __restrict__ tpre,
                                                       int nreg, u64 ntiles, u32 TILE, u32* __restrict__ cnt_t) {
    __shared__ u32 h[4 * 256];
    const int tid = threadIdx.x, wave = tid >> 6;
    for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        for (int i = tid; i < 4 * 256; i += kBlock) h[i] = 0;
        __syncthreads();
        u64 lo, hi;
        rp_tile_range(rstart, tpre, nreg, t, TILE, &lo, &hi);
        u32* hw = h + wave * 256;
        if (digs) {
            // 16-byte loads from the first 16-byte aligned address on
            const u64 alo = min(hi, lo + ((16u - (u32)((uintptr_t)(digs + lo) & 15u)) & 15u));
            for (u64 i = lo + tid; i < alo; i += kBlock) atomicAdd(&hw[digs[i]], 1u);
            const u64 ahi = alo + ((hi - alo) & ~15ull);
            for (u64 i = alo + 16 * (u64)tid; i < ahi; i += 16 * (u64)kBlock) {
                const v4u v = __builtin_nontemporal_load((const v4u*)(digs + i));
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const u32 x = c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
                    atomicAdd(&hw[x & 255u], 1u);
                    atomicAdd(&hw[(x >> 8) & 255u], 1u);
                    atomicAdd(&hw[(x >> 16) & 255u], 1u);
                    atomicAdd(&hw[x >> 24], 1u);
                }
            }
            for (u64 i = ahi + tid; i < hi; i += kBlock) atomicAdd(&hw[digs[i]], 1u);
        } else {
            for (u64 i = lo + tid; i < hi; i += kBlock)
                atomicAdd(&hw[(u32)(__builtin_nontemporal_load(w0 + i) >> shift) & 255u], 1u);
        }
        __syncthreads();
        cnt_t[t * 256 + tid] = h[tid] + h[256 + tid] + h[512 + tid] + h[768 + tid];
        __syncthreads();
    }
}

// KC_RP_ABL (timing ablations of tools/rp_bench, variant builds only): bit 1
// no global stores, bit 2 no ranking / LDS scatter, bit 4 no global loads
#ifndef KC_RP_ABL
#define KC_RP_ABL 0
#endif

template <int NW, bool PAY>
__global__ __launch_bounds__(kRpBlock) void rp_scatter_k(const u64* __restrict__ kin, u64 istride,
                                                         u64* __restrict__ kout, u64 ostride,
                                                         const u32* __restrict__ pin, u32* __restrict__ pout,
                                                         const u64* __restrict__ rstart, const u64* __restrict__ tpre,
                                                         int nreg, u64 ntiles, const u64* __restrict__ pos,
                                                         int dshift, unsigned char* __restrict__ emit, int eshift) {
    constexpr int KPT = RpCfg<NW, PAY>::KPT;
    constexpr int TILE = RpCfg<NW, PAY>::TILE;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64* skey = (u64*)smem;                                    // NW x TILE
    u32* spay = (u32*)(skey + (size_t)NW * TILE);              // TILE (PAY)
    u32* wc = spay + (PAY ? TILE : 0);                         // kRpWaves x 128 words: two u16 counters each
    unsigned short* woff = (unsigned short*)(wc + kRpWaves * 128);  // kRpWaves x 256
    u32* dst = (u32*)(woff + kRpWaves * 256);                        // 256 digit starts in the tile
    u64* gpos = (u64*)(dst + 256);                             // 256 global run starts
    u32* wsum = (u32*)(gpos + 256);                            // 16
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    u64 nk[KPT][NW];
    u32 np[KPT];
    // tiles: with a grid of 8k workgroups, XCD x (blocks b = x mod 8) walks
    // the x-th eighth of the tiles, 8k/8 consecutive tiles at a time, so the
    // digit runs that land next to each other in the output are written
    // through the same L2 (partial lines merge there); else block b walks
    // b, b + grid, ...
    const bool xcd_map = (gridDim.x & 7u) == 0u && ntiles >= 8;
    const u64 step = xcd_map ? (u64)(gridDim.x >> 3) : (u64)gridDim.x;
    const u64 tx = (ntiles + 7) >> 3;
    const u64 t_first = xcd_map ? (u64)(blockIdx.x & 7u) * tx + (blockIdx.x >> 3) : (u64)blockIdx.x;
    const u64 t_end = xcd_map ? min(ntiles, (u64)((blockIdx.x & 7u) + 1) * tx) : ntiles;
    auto load = [&](u64 t) {
        if (t >= t_end) return;
        u64 lo = 0, hi = 0;
        rp_tile_range(rstart, tpre, nreg, t, TILE, &lo, &hi);
        // unconditional loads (clamped into the tile, which is never empty):
        // a per-element select on a load makes hipcc wait for each one
#pragma unroll
        for (int i = 0; i < KPT; i++) {
            const u64 q = min(lo + (u64)i * kRpBlock + tid, hi - 1);
            if (istride == 0) {  // AoS items (uniform branch)
                if constexpr (NW == 2) {
                    const v2u64 v = __builtin_nontemporal_load((const v2u64*)(kin + 2 * q));
                    nk[i][0] = v.x;
                    nk[i][1] = v.y;
                } else {
#pragma unroll
                    for (int j = 0; j < NW; j++) nk[i][j] = __builtin_nontemporal_load(kin + q * NW + j);
                }
            } else {
#pragma unroll
                for (int j = 0; j < NW; j++)
                    nk[i][j] = (KC_RP_ABL & 4) ? (q + 1) * 0x9e3779b97f4a7c15ull * (j + 1)
                                               : __builtin_nontemporal_load(kin + (u64)j * istride + q);
            }
            if constexpr (PAY) np[i] = (KC_RP_ABL & 4) ? (u32)q : __builtin_nontemporal_load(pin + q);
        }
    };
    load(t_first);
    // this tile's 256 global run starts, loaded one tile ahead like the items
    u64 npos = (tid < 256 && t_first < t_end) ? pos[t_first * 256 + tid] : 0ull;
    for (u64 t = t_first; t < t_end; t += step) {
        u64 lo, hi;
        rp_tile_range(rstart, tpre, nreg, t, TILE, &lo, &hi);
        const u32 len = (u32)(hi - lo);
        u64 key[KPT][NW];
        u32 pv[KPT];
#pragma unroll
        for (int i = 0; i < KPT; i++) {
#pragma unroll
            for (int j = 0; j < NW; j++) key[i][j] = nk[i][j];
            pv[i] = PAY ? np[i] : 0u;
        }
        for (int i = tid; i < kRpWaves * 128; i += kRpBlock) wc[i] = 0;
        if (tid < 256) gpos[tid] = npos;
        __syncthreads();
        load(t + step);
        if (tid < 256 && t + step < t_end) npos = pos[(t + step) * 256 + tid];
        u32 rank[KPT];
#pragma unroll
        for (int i = 0; i < KPT; i++) {
            const u32 q = (u32)i * kRpBlock + (u32)tid;
            rank[i] = 0;
            if (q < len && !(KC_RP_ABL & 2)) {
                const u32 d = (u32)(key[i][0] >> dshift) & 255u;
                const u32 sh = 16 * (d & 1);
                rank[i] = (atomicAdd(&wc[wave * 128 + (d >> 1)], 1u << sh) >> sh) & 0xffffu;
            }
        }
        __syncthreads();
        if (tid < 256) {
            u32 run = 0;
            for (int w = 0; w < kRpWaves; w++) {
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
            const u32 q = (u32)i * kRpBlock + (u32)tid;
            if (q < len && !(KC_RP_ABL & 2)) {
                const u32 d = (u32)(key[i][0] >> dshift) & 255u;
                const u32 at = dst[d] + woff[wave * 256 + d] + rank[i];
#pragma unroll
                for (int j = 0; j < NW; j++) skey[(size_t)j * TILE + at] = key[i][j];
                if constexpr (PAY) spay[at] = pv[i];
            }
        }
        __syncthreads();
        for (u32 q = tid; q < len; q += kRpBlock) {
            const u64 k0 = skey[q];
            const u32 d = (u32)(k0 >> dshift) & 255u;
            const u64 g = gpos[d] + (q - dst[d]);
            if (KC_RP_ABL & 1) {
                if (g == ~0ull) kout[0] = k0;  // keeps the work, writes nothing
                continue;
            }
            if (ostride == 0) {  // AoS output (uniform branch)
                if constexpr (NW == 2) {
                    v2u64 v;
                    v.x = k0;
                    v.y = skey[(size_t)TILE + q];
                    *(v2u64*)(kout + 2 * g) = v;
                } else {
                    kout[g * NW] = k0;
#pragma unroll
                    for (int j = 1; j < NW; j++) kout[g * NW + j] = skey[(size_t)j * TILE + q];
                }
            } else {
                kout[g] = k0;
#pragma unroll
                for (int j = 1; j < NW; j++) kout[(u64)j * ostride + g] = skey[(size_t)j * TILE + q];
            }
            if constexpr (PAY) pout[g] = spay[q];
            if (emit) emit[g] = (unsigned char)(k0 >> eshift);
        }
        __syncthreads();
    }
}

static size_t rp_scatter_lds(int NW, bool pay) {
    const size_t tile = (size_t)rp_tile(NW, pay);
    return (size_t)NW * tile * 8 + (pay ? tile * 4 : 0) + kRpWaves * 128 * 4 + kRpWaves * 256 * 2 + 256 * 4 +
           256 * 8 + 16 * 4 + 16;
}

u64* rp_digit_base(u64* tmp, uint64_t ntiles) {
    const u64 nchunks = (ntiles + kP3Chunk - 1) / kP3Chunk;
    return tmp + (ntiles * 256 + 1) / 2 + nchunks * 256;
}

hipError_t launch_rp_hist(const uint8_t* digs, const uint64_t* w0, int shift, const uint64_t* rstart,
                          const uint64_t* tpre, int nreg, uint64_t ntiles, uint32_t tile, uint64_t* pos,
                          uint64_t* tmp, int grid, hipStream_t s) {
    if (ntiles == 0) return hipSuccess;
    u32* cnt_t = (u32*)tmp;
    u64* csum = tmp + (ntiles * 256 + 1) / 2;
    const u64 nchunks = (ntiles + kP3Chunk - 1) / kP3Chunk;
    u64* dtot = csum + nchunks * 256;
    const int gu = (int)hmin(ntiles, (u64)grid * 4);
    hipLaunchKernelGGL(rp_upsweep_k, dim3(gu), dim3(kBlock), 0, s, (const unsigned char*)digs, w0, shift, rstart,
                       tpre, nreg, ntiles, tile, cnt_t);
    hipLaunchKernelGGL(p3_chunk_sum_k, dim3(nchunks), dim3(256), 0, s, (const u32*)cnt_t, ntiles, csum);
    hipLaunchKernelGGL(p3_chunk_scan_k, dim3(256), dim3(256), 0, s, csum, nchunks, dtot);
    hipLaunchKernelGGL(p3_digit_base_k, dim3(1), dim3(256), 0, s, dtot);
    hipLaunchKernelGGL(p3_chunk_pos_k, dim3(nchunks), dim3(256), 0, s, (const u32*)cnt_t, (const u64*)csum,
                       (const u64*)dtot, ntiles, pos);
    return hipGetLastError();
}

// MSD form of the regional histogram: digit runs are placed inside their
// region (region start + the region's smaller digits + the region's earlier
// tiles), so a pass sorts every region by the digit and regions stay in
// order (the rp_hist passes above are LSD: digit-major over all regions).
// One 256-thread workgroup (one thread per digit) per region.
__global__ __launch_bounds__(256) void rp_region_pos_k(const u32* __restrict__ cnt_t, const u64* __restrict__ rstart,
                                                       const u64* __restrict__ tpre, u32 nreg, u64* __restrict__ pos) {
    __shared__ u64 part[256];
    const int d = threadIdx.x;
    for (u32 r = blockIdx.x; r < nreg; r += gridDim.x) {
        const u64 t0 = tpre[r], t1 = tpre[r + 1];
        u64 sum = 0;
        for (u64 t = t0; t < t1; t++) sum += cnt_t[t * 256 + d];
        part[d] = sum;
        __syncthreads();
        // exclusive scan over the 256 digits (Hillis-Steele in LDS)
        for (int o = 1; o < 256; o <<= 1) {
            const u64 y = d >= o ? part[d - o] : 0ull;
            __syncthreads();
            part[d] += y;
            __syncthreads();
        }
        u64 run = rstart[r] + part[d] - sum;
        for (u64 t = t0; t < t1; t++) {
            pos[t * 256 + d] = run;
            run += cnt_t[t * 256 + d];
        }
        __syncthreads();
    }
}

hipError_t launch_rp_hist_regional(const uint64_t* w0, int shift, const uint64_t* rstart, const uint64_t* tpre,
                                   int nreg, uint64_t ntiles, uint32_t tile, uint64_t* pos, uint32_t* cnt_t, int grid,
                                   hipStream_t s, const uint8_t* digs) {
    if (ntiles == 0) return hipSuccess;
    const int gu = (int)hmin(ntiles, (u64)grid * 4);
    // digs: the digit byte of every item, written by the pass that placed
    // them (1 B read per item instead of word 0)
    hipLaunchKernelGGL(rp_upsweep_k, dim3(gu), dim3(kBlock), 0, s, (const unsigned char*)digs, digs ? nullptr : w0,
                       shift, rstart, tpre, nreg, ntiles, tile, cnt_t);
    hipLaunchKernelGGL(rp_region_pos_k, dim3((u32)hmin((u64)nreg, 65536)), dim3(256), 0, s, (const u32*)cnt_t, rstart,
                       tpre, (u32)nreg, pos);
    return hipGetLastError();
}

hipError_t launch_rp_scatter(int NW, bool pay, const uint64_t* kin, uint64_t istride, uint64_t* kout,
                             uint64_t ostride, const uint32_t* pin, uint32_t* pout, const uint64_t* rstart,
                             const uint64_t* tpre, int nreg, uint64_t ntiles, const uint64_t* pos, int dshift,
                             uint8_t* emit, int eshift, int grid, hipStream_t s) {
    if (ntiles == 0) return hipSuccess;
    // one persistent workgroup per CU (the LDS tile allows no second one): a
    // larger grid would run as two rounds of workgroups, each restarting its
    // prefetch pipeline
    const int g = (int)hmin(ntiles, (u64)(grid / 2 > 0 ? KC_RP_WPC * grid / 2 : 1));
    const size_t lds = (rp_scatter_lds(NW, pay) + 15) & ~(size_t)15;
#define KC_RPS(NWV, PAYV)                                                                                          \
    hipLaunchKernelGGL((rp_scatter_k<NWV, PAYV>), dim3(g), dim3(kRpBlock), lds, s, kin, istride, kout, ostride, pin, \
                       pout, rstart, tpre, nreg, ntiles, pos, dshift, (unsigned char*)emit, eshift)
    if (pay) {
        switch (NW) {
        case 1: KC_RPS(1, true); break;
        case 2: KC_RPS(2, true); break;
        case 3: KC_RPS(3, true); break;
        case 4: KC_RPS(4, true); break;
        default: return hipErrorInvalidValue;
        }
    } else {
        switch (NW) {
        case 1: KC_RPS(1, false); break;
        case 2: KC_RPS(2, false); break;
        case 3: KC_RPS(3, false); break;
        case 4: KC_RPS(4, false); break;
        default: return hipErrorInvalidValue;
        }
    }
#undef KC_RPS
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// P5 of the skm engine: count_buckets over records. Each wave expands its 64
// records (one per lane) into a flat key sequence: an exclusive scan of the
// key counts, then rounds of 64 keys in which a scalar loop walks the owner
// records of the round (v_readlane broadcasts) and every lane picks the key
// at its position. Keys then take the LDS table exactly as in count_buckets
// (home-group fast path, per-wave slow-path queue of (record, key index),
// sub-range passes, global table and spill at the last level).
// ---------------------------------------------------------------------------

struct SkmBucketArgs {
    const u64* recs;  // RW x stride (SoA), grouped by bucket
    u64 stride;
    const u64* starts;
    u32 b0, nbuckets;  // buckets [b0, nbuckets)
    u32 lcap;
    int count_keys;
    u64 last_mask;
    u64* rec_keys;
    u32* rec_cnts;
    unsigned char* rec_dig;  // may be null: each record's word 0 bits 48..55 (the finish's first digit)
    u64 rec_cap;
    u64* rec_cursor;
    u64* table;
    u64 cap;
    u64* spill;
    u64 spill_cap;
    u64* spill_ctr;
    u64* stats;
    u32 probe_limit;
    int skip;
    // deduplicated records (P5a, count_rec_k): bucket b's dlen[b] distinct
    // records at the front of its own range with their multiplicities dcnt
    // (indexed like recs); dlen == nullptr or dlen[b] == kRawList: the
    // bucket's own records (multiplicity 1)
    const u32* dcnt;
    const u32* dlen;
    const u64* dpos;  // kOverList buckets: their list's start
};

constexpr u32 kRawList = 0xffffffffu;  // P5a: bucket not deduplicated
constexpr u32 kOverList = 0x80000000u;  // P5a: dlen flag, the list is at dpos[b] (overflow list), not at the bucket's start

// key i of a record (see the record layout above)
template <int W>
__device__ __forceinline__ void skm_key(const u64 (&rw)[W + 1], u32 i, u64 last_mask, u64 (&key)[W]) {
    const u32 o = 16u + 2u * i;
    const bool hiw = o >= 64u;
    const u32 sh = o & 63u;
    u64 ext[W + 2];
#pragma unroll
    for (int j = 0; j <= W; j++) ext[j] = rw[j];
    ext[W + 1] = 0ull;
#pragma unroll
    for (int j = 0; j < W; j++) {
        const u64 a0 = hiw ? ext[j + 1] : ext[j];
        const u64 a1 = hiw ? ext[j + 2] : ext[j + 1];
        key[j] = sh ? ((a0 << sh) | (a1 >> (64u - sh))) : a0;
    }
    key[W - 1] &= last_mask;
}

constexpr int kSkmGroup = 4;    // P5 LDS table: slots per group (two 16-byte loads per key)
#ifndef KC_P5_CLAIM
#define KC_P5_CLAIM 1  // P5 (W = 1): new keys claim an empty home-group slot in the walk, not the slow path
#endif
constexpr u32 kSkmQueue = 128;  // P5 per-wave slow-path queue entries (u64: key at W = 1, else record << 6 | key index)

// P5 LDS: table (lcap slots) + misc (48 u32) + per-wave slow-path queues +
// per-wave record stage (64 records of W + 1 words + one spare, so the record
// after the last can be read unconditionally)
// (+ per-wave u32 weights of the queue and of the record stage)
static size_t skm_fixed_lds(int W) {
    return 48 * 4 + (size_t)kBucketWaves * kSkmQueue * 8 + (size_t)kBucketWaves * 65 * (W + 1) * 8 +
           (size_t)kBucketWaves * (kSkmQueue + 65) * 4 + 16;
}

int skm_lds_slots(int W) {
    const int per = 8 * W + 4 + (W >= 2 ? 4 : 0);
    const int slots = (int)((160 * 1024 - 64 - skm_fixed_lds(W)) / per);
    return slots / 64 * 64;
}

static size_t skm_bucket_lds_bytes(int W) {
    const size_t lcap = (size_t)skm_lds_slots(W);
    return lcap * (8 * W + 4 + (W >= 2 ? 4 : 0)) + skm_fixed_lds(W);
}

// bases of a record from bit offset o (16 + 2 * key index) as RW words, base
// o at the top, zeros past the record
template <int RW>
__device__ __forceinline__ void skm_window(const u64 (&rec)[RW], u32 o, u64 (&win)[RW]) {
    const bool hiw = o >= 64u;
    const u32 sh = o & 63u;
    u64 ext[RW + 2];
#pragma unroll
    for (int j = 0; j < RW; j++) ext[j] = rec[j];
    ext[RW] = 0ull;
    ext[RW + 1] = 0ull;
#pragma unroll
    for (int j = 0; j < RW; j++) {
        const u64 a0 = hiw ? ext[j + 1] : ext[j];
        const u64 a1 = hiw ? ext[j + 2] : ext[j + 1];
        win[j] = sh ? ((a0 << sh) | (a1 >> (64u - sh))) : a0;
    }
}

// 32-bit slot hash of a key (P5 of the skm engine): the LDS group of a key is
// umulhi(h, groups); lds_insert takes the same position as the 48-bit
// fraction h << 16
template <int W>
__device__ __forceinline__ u32 skm_hash32(const u64 (&key)[W]) {
    u64 x = key[0];
#pragma unroll
    for (int j = 1; j < W; j++) x = (x ^ (x >> 29)) * 0xc2b2ae3d27d4eb4full + key[j];
    x ^= x >> 31;
    return ((u32)x ^ (u32)(x >> 32)) * 0x9e3779b1u;
}

struct SkmLdsTable {
    u64* lkeys;
    u32* lcnt;
    u32* lstate;
    u32* lfill;
    u32* labort;
};

// Slow path for the first c entries of a wave's queue (the key itself at
// W = 1, else record << 6 | key index):
// full probing insert into the LDS table, fill/abort accounting, and at the
// last sub-range level the global table and the spill buffer. Out of line:
// it runs once per 64 queued keys and keeps the hot loop small.
template <int W>
__device__ __forceinline__ void skm_drain(const SkmBucketArgs& a, SkmLdsTable t, const u64* wq, const u32* wqw, u32 c,
                                       const u64* recs, u64 stride, u64 lo, bool last, u32 limit) {
    constexpr int RW = W + 1;
    const int lane = (int)lane_id();
    const bool act = lane < (int)c;
    u64 qk[W];
#pragma unroll
    for (int j = 0; j < W; j++) qk[j] = 0;
    const u32 w = act ? wqw[lane] : 0u;  // the key's multiplicity
    if (act) {
        const u64 e = wq[lane];
        if constexpr (W == 1) {
            qk[0] = e;  // W = 1 queues the key itself
        } else {
            const u64 ri = lo + (e >> 6);
            u64 rw[RW];
#pragma unroll
            for (int j = 0; j < RW; j++) rw[j] = recs[(u64)j * stride + ri];
            skm_key<W>(rw, (u32)(e & 63u), a.last_mask, qk);
        }
    }
    bool done = true, claimed = false, lclaim = false, full = false;
    if (act) {
        const u64 frac = (u64)skm_hash32<W>(qk) << 16;
        if (!lds_insert<W, kSkmGroup>(qk, frac, t.lkeys, t.lcnt, t.lstate, a.lcap,
                                      last ? a.lcap : (a.lcap < 64u ? a.lcap : 64u), &lclaim, w)) {
            if (!last) {
                full = true;
            } else if constexpr (W == 1) {
                done = insert_w1(qk[0], a.table, a.cap, a.probe_limit, &claimed, w);
            } else {
                done = insert_wide<W>(qk, a.table, a.cap, a.probe_limit, &claimed, w);
            }
        }
    }
    // lfill counts the pass's claimed slots (= its records at the emission)
    const u64 lm = __ballot(lclaim);
    const u64 fm = __ballot(full);
    if ((lm || fm) && lane == 0) {
        u32 f = atomicAdd(t.lfill, (u32)__popcll(lm)) + (u32)__popcll(lm);
        if (!last && (fm || f > limit)) atomicOr(t.labort, 1u);
    }
    if (last) {
        u64 cm = __ballot(claimed);
        if (cm && lane == __ffsll((long long)cm) - 1)
            atomicAdd((unsigned long long*)&a.stats[ST_CLAIMED], (unsigned long long)__popcll(cm));
        // a spilled key is written once per unit of its multiplicity (the
        // spill runs are counted by sort + run length)
        const u32 ws = done ? 0u : w;
        if (__ballot(ws != 0u)) {
            const u32 inc = wave_incl_scan(ws);
            const u32 tot = (u32)__builtin_amdgcn_readlane((int)inc, 63);
            u64 base = 0;
            if (lane == 0) base = atomicAdd((unsigned long long*)a.spill_ctr, (unsigned long long)tot);
            base = readlane64(base, 0);
            const u64 idx = base + (inc - ws);
            for (u32 r = 0; r < ws; r++) {
                if (idx + r < a.spill_cap) {
#pragma unroll
                    for (int j = 0; j < W; j++) a.spill[(u64)j * a.spill_cap + idx + r] = qk[j];
                } else {
                    atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_SPILL_OVERFLOW);
                }
            }
        }
    }
}

// starts_r / dlen_r: a.starts / a.dlen as read-only kernel arguments, so the
// per-bucket ranges are scalar loads (lgkmcnt), which never wait behind the
// vector loads of records in flight (in-order vmcnt)
template <int W>
__global__ __launch_bounds__(kBucketBlock) void count_skm_k(SkmBucketArgs a, const u64* __restrict__ starts_r,
                                                           const u32* __restrict__ dlen_r) {
    constexpr int RW = W + 1;
    constexpr int PD = 2;  // record batches in flight
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64* lkeys = (u64*)smem;                         // W x lcap
    u32* lcnt = (u32*)(lkeys + (size_t)W * a.lcap);  // lcap
    u32* lstate = lcnt + a.lcap;                     // lcap (W >= 2)
    u32* misc = lstate + (W >= 2 ? a.lcap : 0);      // base (2 @16), fill, abort, next, kscan, wave totals (16 @24)
    u32* lfill = misc + 20;
    u32* labort = misc + 21;
    u32* lnext = misc + 22;
    u32* lkscan = misc + 23;  // keys of an aborted pass scanned (abort estimate)
    const int tid = threadIdx.x;
    const int lane = (int)lane_id();
    const u64 lane_lt = lanemask_lt();
    u64* wq = (u64*)(misc + 48) + (tid >> 6) * kSkmQueue;
    u64* wst = (u64*)(misc + 48) + kBucketWaves * kSkmQueue + (tid >> 6) * 65 * RW;  // this wave's record stage (+1 spare)
    u32* wqw = (u32*)((u64*)(misc + 48) + kBucketWaves * kSkmQueue + kBucketWaves * 65 * RW) +
               (tid >> 6) * kSkmQueue;                                  // queue multiplicities
    u32* wsw = (u32*)((u64*)(misc + 48) + kBucketWaves * kSkmQueue + kBucketWaves * 65 * RW) +
               kBucketWaves * kSkmQueue + (tid >> 6) * 65;              // stage multiplicities
    const SkmLdsTable tab = {lkeys, lcnt, lstate, lfill, labort};
    for (u32 i = tid; i < a.lcap; i += kBucketBlock) {
#pragma unroll
        for (int j = 0; j < W; j++) lkeys[(size_t)j * a.lcap + i] = 0ull;
        lcnt[i] = 0;
        if constexpr (W >= 2) lstate[i] = 0;
    }
    if (tid == 0) {
        *lfill = 0;
        *labort = 0;
        *lkscan = 0;
    }
    __syncthreads();
    const u32 limit = (a.lcap * 13u) >> 4;
    const u32 mmax = a.lcap >= 64 ? kMaxSub : 1u;
    const u32 ng = a.lcap / kSkmGroup;
    const bool grouped = W == 1 && (a.lcap % kSkmGroup) == 0;
    // the first PD batches of a pass are loaded while the previous pass ends
    // (speculatively the next bucket's; a sub-range pass of the same bucket
    // reloads): pfb is the bucket pf holds the pass-start batches of
    u64 pf[PD][RW];
    u32 pfw[PD];
    u32 pfb = ~0u;
    // bucket bb's record source: deduplicated list or its own records
    auto source = [&](u32 bb, const u64** rp, u64* st, const u32** cp, u64* l0, u64* h0) {
        const u32 dl = dlen_r ? dlen_r[bb] : kRawList;
        if (dl != kRawList) {
            *rp = a.recs;
            *st = a.stride;
            *cp = a.dcnt;
            *l0 = (dl & kOverList) ? a.dpos[bb] : starts_r[bb];  // overflow list: in the pool's tail
            *h0 = *l0 + (dl & ~kOverList);
        } else {
            *rp = a.recs;
            *st = a.stride;
            *cp = nullptr;
            *l0 = starts_r[bb];
            *h0 = starts_r[bb + 1];
        }
    };
    auto prefetch_pass = [&](u32 bb) {
        const u64* rp;
        u64 rst, l0, h0;
        const u32* cp;
        source(bb, &rp, &rst, &cp, &l0, &h0);
        const u64 nr0 = h0 - l0, pw = (nr0 + kBucketWaves - 1) / kBucketWaves;
        const u64 w0 = l0 + min(nr0, (u64)(tid >> 6) * pw), w1 = l0 + min(nr0, (u64)((tid >> 6) + 1) * pw);
#pragma unroll
        for (int d = 0; d < PD; d++) {
            const u64 i = w0 + (u64)d * 64 + lane;
#pragma unroll
            for (int j = 0; j < RW; j++) pf[d][j] = i < w1 ? rp[(u64)j * rst + i] : 0ull;
            pfw[d] = (cp && i < w1) ? cp[i] : 1u;
        }
        pfb = bb;
    };
    // the record-overflow flag, read one bucket ahead (its latency hidden by
    // the bucket's work; a late stop only costs records the host rewrites)
    if (a.skip & 8) return;  // timing experiments: launch only
    // A global load waits for every older load of its wave (in-order vmcnt),
    // so nothing here waits on a global value while the next bucket's records
    // are in flight: the record-overflow flag (an early stop only saves work;
    // records past rec_cap are never written and the host reruns) is read
    // every 64 buckets, and the output range is reserved before the prefetch.
    u32 nb_done = 0;
    for (u32 b = a.b0 + blockIdx.x; b < a.nbuckets; b += gridDim.x, nb_done++) {
        if ((nb_done & 63u) == 0u) {
            if (tid == 0)
                *lnext = (u32)(__hip_atomic_load((unsigned long long*)&a.stats[ST_ERR], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) &
                               ERR_REC_OVERFLOW);
            __syncthreads();
            const bool stop = *lnext != 0u;
            __syncthreads();
            if (stop) return;
        }
        const u64* brecs;
        u64 bstride, lo, hi;
        const u32* bcnt;
        source(b, &brecs, &bstride, &bcnt, &lo, &hi);
        if (a.count_keys) {
            u64 kn = 0;
            for (u64 i = lo + tid; i < hi; i += kBucketBlock)
                kn += (brecs[(u64)(RW - 1) * bstride + i] & 63u) * (u64)(bcnt ? bcnt[i] : 1u);
            wave_add(&a.stats[ST_P5_KEYS], kn);
        }
        u32 m = 1, sub = 0;
        while (sub < m) {
            const bool last = m >= mmax;
            // sub-range of a key: bits [48 - log2 m, 48) (m is a power of two),
            // = ((key & M48) * m) >> 48 as in count_buckets
            const u32 msh = 48u - (31u - (u32)__builtin_clz(m));
            u64 scanned = 0;
            u32 my_keys = 0;
            u32 qn = 0;
            // every wave takes an equal contiguous share of the bucket's
            // records, 64 at a time (no wave idles through a short last batch);
            // the records of its next PD batches (one per lane) are in flight
            const u64 nrec_b = hi - lo;
            const u64 per_w = (nrec_b + kBucketWaves - 1) / kBucketWaves;
            const u64 wlo = lo + min(nrec_b, (u64)(tid >> 6) * per_w), whi = lo + min(nrec_b, (u64)((tid >> 6) + 1) * per_w);
            if (pfb != b) prefetch_pass(b);
            pfb = ~0u;
            for (u64 base = wlo; base < whi; base += 64) {
                if (!last && __hip_atomic_load(labort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                scanned += 64;
                // this batch's record -> the wave's LDS stage; next loads issued
#pragma unroll
                for (int j = 0; j < RW; j++) wst[(size_t)lane * RW + j] = pf[0][j];
                wsw[lane] = pfw[0];
                const u32 n = (u32)(pf[0][RW - 1] & 63u);
#pragma unroll
                for (int d = 0; d + 1 < PD; d++) {
#pragma unroll
                    for (int j = 0; j < RW; j++) pf[d][j] = pf[d + 1][j];
                    pfw[d] = pfw[d + 1];
                }
                {
                    const u64 i = base + (u64)PD * 64 + lane;
#pragma unroll
                    for (int j = 0; j < RW; j++) pf[PD - 1][j] = i < whi ? brecs[(u64)j * bstride + i] : 0ull;
                    pfw[PD - 1] = (bcnt && i < whi) ? bcnt[i] : 1u;
                }
                // the wave's keys as one flat sequence: exclusive scan of the
                // records' key counts; lane l takes keys [l*per, l*per + per)
                u32 inc = n;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const u32 y = __shfl_up(inc, o);
                    if (lane >= o) inc += y;
                }
                const u32 excl = inc - n;
                const u32 T = (u32)__builtin_amdgcn_readlane((int)inc, 63);
                if (T == 0 || (a.skip & 4)) continue;
                const u32 per = (a.skip & 2) ? 0u : (T + 63) >> 6;
                const u32 s0 = min(T, (u32)lane * per), s1 = min(T, s0 + per);
                // owner of key s0: the last record whose first key is <= s0
                int o = 0;
#pragma unroll
                for (int st = 32; st >= 1; st >>= 1) {
                    const u32 e = (u32)__shfl((int)excl, o + st);
                    if (e <= s0) o += st;
                }
                u32 ki = s0 - (u32)__shfl((int)excl, o);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
                __builtin_amdgcn_wave_barrier();
                u64 cur[RW];
#pragma unroll
                for (int j = 0; j < RW; j++) cur[j] = wst[(size_t)o * RW + j];
                u32 wcur = wsw[o];  // the current record's multiplicity
                u32 nn = (u32)(cur[RW - 1] & 63u);
                u64 win[RW];
                skm_window<RW>(cur, 16u + 2u * ki, win);
                const u64 wrec0 = base - lo;  // lane 0's record of this batch
                // advance to the next key: roll one base in; past the record's
                // last key move to the next record with keys (this wave's stage)
                // the record after the current one waits in registers (nxt),
                // so a switch costs no LDS round trip
                u64 nxt[RW];
#pragma unroll
                for (int j = 0; j < RW; j++) nxt[j] = wst[(size_t)(o + 1) * RW + j];
                u32 wnxt = wsw[o + 1];
                auto advance = [&](u32 t) {
#pragma unroll
                    for (int j = 0; j < RW - 1; j++) win[j] = (win[j] << 2) | (win[j + 1] >> 62);
                    win[RW - 1] <<= 2;
                    ++ki;
                    if (ki == nn && s0 + t + 1 < s1) {
                        ++o;
#pragma unroll
                        for (int j = 0; j < RW; j++) cur[j] = nxt[j];
                        wcur = wnxt;
                        // every record of a counted bucket has n >= 1: F writes
                        // n = 0 padding only into bucket 0xffff, never counted
                        nn = (u32)(cur[RW - 1] & 63u);
                        skm_window<RW>(cur, 16u, win);
                        // unconditional (spare record past the last) and issued
                        // after cur's last use, into nxt's own registers: the value
                        // is needed only at the next switch, so no wait here
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int j = 0; j < RW; j++) nxt[j] = wst[(size_t)(o + 1) * RW + j];
                        wnxt = wsw[o + 1];
                        ki = 0;
                    }
                };
                if (W == 1 && grouped) {
                    u32 fclaim = 0;  // slots this lane claimed in this batch
                    // software pipeline: the home group of key t + 1 is loaded
                    // while key t is resolved (a group read before a claim of
                    // the slow path only sends that key to the slow path again)
                    u64 key = win[0] & a.last_mask;
                    u32 kw = wcur;
                    bool act = s0 < s1;
                    // (group halves swizzled: logical slot j at kSkmGroup g + (j ^ gswz(g)))
                    u32 g = __umulhi(skm_hash32<1>(*(const u64(*)[1])&key), ng);
                    v2u64 a0 = *(const lds_v2u64*)(lkeys + kSkmGroup * g + gswz(g));
                    v2u64 a1 = *(const lds_v2u64*)(lkeys + kSkmGroup * g + (2u ^ gswz(g)));
                    for (u32 t = 0; t < per; t++) {
                        advance(t);
                        const bool act_n = s0 + t + 1 < s1;
                        const u64 key_n = win[0] & a.last_mask;
                        const u32 kw_n = wcur;
                        const u32 g_n = __umulhi(skm_hash32<1>(*(const u64(*)[1])&key_n), ng);
                        const v2u64 b0 = *(const lds_v2u64*)(lkeys + kSkmGroup * g_n + gswz(g_n));
                        const v2u64 b1 = *(const lds_v2u64*)(lkeys + kSkmGroup * g_n + (2u ^ gswz(g_n)));
                        bool want = act && !a.skip;
                        want = want && ((u32)(key >> msh) & (m - 1u)) == sub;
                        my_keys += want ? 1u : 0u;
                        // a key sits in at most one slot and is never 0 (key 0^W
                        // is counted outside the table), so any equal slot is it
                        const bool e0 = a0.x == key, e1 = a0.y == key, e2 = a1.x == key, e3 = a1.y == key;
                        const int hit = e0 ? 0 : (e1 ? 1 : (e2 ? 2 : 3));
                        const bool found = want && (e0 || e1 || e2 || e3);
                        if (found) atomicAdd(&lcnt[kSkmGroup * g + ((u32)hit ^ gswz(g))], kw);
                        bool pend = want && !found;
                        if constexpr (KC_P5_CLAIM) {
                            // a new key takes the first empty slot of its home
                            // group here (slots fill in order and never empty
                            // within a pass, so a key still sits in one slot);
                            // a lost race goes to the slow path
                            const bool z0 = a0.x == 0ull, z1 = a0.y == 0ull, z2 = a1.x == 0ull, z3 = a1.y == 0ull;
                            if (pend && (z0 || z1 || z2 || z3)) {
                                const u32 sl = kSkmGroup * g + ((z0 ? 0u : (z1 ? 1u : (z2 ? 2u : 3u))) ^ gswz(g));
                                const u64 old = atomicCAS((unsigned long long*)&lkeys[sl], 0ull, (unsigned long long)key);
                                if (old == 0ull || old == key) {
                                    atomicAdd(&lcnt[sl], kw);
                                    fclaim += old == 0ull ? 1u : 0u;
                                    pend = false;
                                }
                            }
                        }
                        const u64 pb = __ballot(pend);
                        if (pb) {
                            if (pend) {
                                const u32 at = qn + (u32)__popcll(pb & lane_lt);
                                wq[at] = key;
                                wqw[at] = kw;
                            }
                            qn += (u32)__popcll(pb);
                            if (qn >= 64) {
                                skm_drain<W>(a, tab, wq, wqw, 64, brecs, bstride, lo, last, limit);
                                const u32 rest = qn - 64;
                                const u64 keep = lane < (int)rest ? wq[64 + lane] : 0ull;
                                const u32 keepw = lane < (int)rest ? wqw[64 + lane] : 0u;
                                if (lane < (int)rest) {
                                    wq[lane] = keep;
                                    wqw[lane] = keepw;
                                }
                                qn = rest;
                            }
                        }
                        key = key_n;
                        kw = kw_n;
                        act = act_n;
                        g = g_n;
                        a0 = b0;
                        a1 = b1;
                    }
                    if constexpr (KC_P5_CLAIM) {
                        // this batch's claims into the pass's fill count (exact
                        // before the emission; the abort check follows it)
                        u32 fc = fclaim;
                        for (int o2 = 32; o2 >= 1; o2 >>= 1) fc += (u32)__shfl_xor((int)fc, o2);
                        if (fc && lane == 0) {
                            const u32 f = atomicAdd(lfill, fc) + fc;
                            if (!last && f > limit) atomicOr(labort, 1u);
                        }
                        fclaim = 0;
                    }
                } else {
                for (u32 t = 0; t < per; t++) {
                    const bool act = s0 + t < s1;
                    u64 key[W];
#pragma unroll
                    for (int j = 0; j < W; j++) key[j] = win[j];
                    key[W - 1] &= a.last_mask;
                    bool want = act && !a.skip;
                    want = want && ((u32)(key[0] >> msh) & (m - 1u)) == sub;
                    my_keys += want ? 1u : 0u;
                    bool found = false;
                    const u32 h = skm_hash32<W>(key);
                    if constexpr (W >= 2) {
                        const u32 sl = __umulhi(h, a.lcap);
                        if (__hip_atomic_load(&lstate[sl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 2u) {
                            bool eq = true;
#pragma unroll
                            for (int j = 0; j < W; j++) eq = eq && lkeys[(size_t)j * a.lcap + sl] == key[j];
                            found = want && eq;
                            if (found) atomicAdd(&lcnt[sl], wcur);
                        }
                    }
                    const bool pend = want && !found;
                    const u64 pb = __ballot(pend);
                    if (pb) {
                        if (pend) {
                            const u32 at = qn + (u32)__popcll(pb & lane_lt);
                            wq[at] = W == 1 ? key[0] : (((wrec0 + (u64)o) << 6) | ki);
                            wqw[at] = wcur;
                        }
                        qn += (u32)__popcll(pb);
                        if (qn >= 64) {
                            skm_drain<W>(a, tab, wq, wqw, 64, brecs, bstride, lo, last, limit);
                            const u32 rest = qn - 64;
                            const u64 keep = lane < (int)rest ? wq[64 + lane] : 0ull;
                            const u32 keepw = lane < (int)rest ? wqw[64 + lane] : 0u;
                            if (lane < (int)rest) {
                                wq[lane] = keep;
                                wqw[lane] = keepw;
                            }
                            qn = rest;
                        }
                    }
                    advance(t);
                }
                }
            }
            // the next bucket's first batches go in flight during the emission
            // (unless another pass of this bucket follows)
            const bool pf_next = sub + 1 >= m && b + gridDim.x < a.nbuckets;
            if (qn && (last || !__hip_atomic_load(labort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
                skm_drain<W>(a, tab, wq, wqw, qn, brecs, bstride, lo, last, limit);
            __syncthreads();
            const bool aborted = *labort != 0u;
            if (aborted && my_keys) atomicAdd(lkscan, my_keys);
            __syncthreads();
            if (aborted) {
                if (tid == 0) {
                    // distinct keys of the bucket, extrapolated from the scanned
                    // fraction f of its records: linear when keys repeat rarely
                    // in the scanned part, ~all seen already when they repeat
                    // often (genome coverage)
                    // (wave 0's share stands for the bucket)
                    const u64 w0n = min(nrec_b, per_w);
                    const float f = (float)min(scanned, w0n) / (float)(w0n ? w0n : 1);
                    const float rep = (float)(*lkscan) / (float)(*lfill ? *lfill : 1u);
                    const float seen = rep >= 4.f ? 1.f : (rep >= 2.f ? fmaxf(f, 0.5f) : fmaxf(f, 1e-6f));
                    const u64 est = (u64)((float)(*lfill) * (float)m / seen);
                    *lkscan = 0;
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
                const u32 nm = *lnext;
                sub *= nm / m;
                m = nm;
                __syncthreads();
                continue;
            }
            {
                const int wave = tid >> 6;
                const u32 spw = (a.lcap + kBucketWaves - 1) / kBucketWaves;
                const u32 s0 = (u32)wave * spw;
                const u32 s1 = min(a.lcap, s0 + spw);
                // the pass's records = its claimed slots: the output range is
                // reserved now, its latency hidden by the waves' slot counts
                if (a.skip & 16) {  // timing experiments: no emission
                    if (pf_next) prefetch_pass(b + gridDim.x);
                    __syncthreads();
                    ++sub;
                    continue;
                }
                // one scan of the table: each wave's occupied slots of a
                // 64-slot chunk take consecutive places from an LDS cursor
                // (record order inside the bucket is free: the finish sorts)
                const u32 nclaimed = *lfill;
                if (tid == 0) {
                    *(u64*)(misc + 16) =
                        nclaimed ? atomicAdd((unsigned long long*)a.rec_cursor, (unsigned long long)nclaimed) : 0ull;
                    misc[24] = 0u;
                }
                if (pf_next) prefetch_pass(b + gridDim.x);
                __syncthreads();
                const u64 rbase = *(const u64*)(misc + 16);
                for (u32 c0 = s0; c0 < s1; c0 += 64) {
                    const u32 i = c0 + (u32)lane;
                    const bool occ = i < s1 && ((W == 1) ? (lkeys[i] != 0ull) : (lstate[i] == 2u));
                    const u64 bm = __ballot(occ);
                    if (bm == 0ull) continue;
                    u32 at = 0;
                    if (lane == 0) at = atomicAdd(&misc[24], (u32)__popcll(bm));
                    at = (u32)__builtin_amdgcn_readfirstlane((int)at);
                    if (occ) {
                        const u64 qq = rbase + at + (u64)__popcll(bm & lane_lt);
                        if (qq < a.rec_cap) {
#pragma unroll
                            for (int j = 0; j < W; j++)
                                a.rec_keys[(u64)j * a.rec_cap + qq] = lkeys[(size_t)j * a.lcap + i];
                            a.rec_cnts[qq] = lcnt[i];
                            if (a.rec_dig) a.rec_dig[qq] = (unsigned char)(lkeys[i] >> 48);
                        }
#pragma unroll
                        for (int j = 0; j < W; j++) lkeys[(size_t)j * a.lcap + i] = 0ull;
                        lcnt[i] = 0;
                        if constexpr (W >= 2) lstate[i] = 0;
                    }
                }
                __syncthreads();
                if (tid == 0) {
                    const u32 total = misc[24];
                    if (rbase + total > a.rec_cap || total != nclaimed)
                        atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_REC_OVERFLOW);
                    *lfill = 0;
                    atomicAdd((unsigned long long*)&a.stats[ST_P5_PASSES], 1ull);
                }
            }
            __syncthreads();
            ++sub;
        }
    }
}

hipError_t launch_count_skm(int W, int k, const uint64_t* recs, uint64_t stride, const uint64_t* starts,
                            uint32_t b0, uint32_t b1, bool count_keys, uint64_t* rec_keys, uint32_t* rec_cnts, uint64_t rec_cap,
                            uint64_t* rec_cursor, uint64_t* table, uint64_t cap, uint64_t* spill, uint64_t spill_cap,
                            uint64_t* stats, uint32_t probe_limit, uint32_t lcap, int grid, hipStream_t s,
                            const SkmDedup* dd, uint8_t* rec_dig) {
    SkmBucketArgs a;
    a.rec_dig = rec_dig;
    a.dcnt = dd ? dd->cnt : nullptr;
    a.dlen = dd ? dd->len : nullptr;
    a.dpos = dd ? dd->pos : nullptr;
    a.skip = experiment_knob("KC_P5_SKIP");
    const bool mask_last = ((k + 3) / 4) < 8 * W;
    a.last_mask = mask_last ? (~0ull << (64 - 2 * (k & 31))) : ~0ull;
    a.recs = recs;
    a.stride = stride;
    a.starts = starts;
    a.b0 = b0;
    a.nbuckets = b1;
    a.count_keys = count_keys ? 1 : 0;
    a.lcap = (lcap == 0 || lcap > (u32)skm_lds_slots(W)) ? (u32)skm_lds_slots(W) : lcap;
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
    const size_t lds = (skm_bucket_lds_bytes(W) + 15) & ~(size_t)15;
    switch (W) {
    case 1: hipLaunchKernelGGL(count_skm_k<1>, dim3(grid), dim3(kBucketBlock), lds, s, a, a.starts, a.dlen); break;
    case 2: hipLaunchKernelGGL(count_skm_k<2>, dim3(grid), dim3(kBucketBlock), lds, s, a, a.starts, a.dlen); break;
    case 3: hipLaunchKernelGGL(count_skm_k<3>, dim3(grid), dim3(kBucketBlock), lds, s, a, a.starts, a.dlen); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}


// ---------------------------------------------------------------------------
// P5a: count_rec_k (W = 1). At genome coverage most super-k-mer records of a
// bucket are copies of one another: every read that covers a run of windows
// sharing one minimizer cuts the same record (only runs cut by a read end or a
// bad base differ). Each workgroup takes buckets like P5; the bucket's records
// go into an LDS table of whole records (both words; the bucket bits replaced
// by a non-zero marker, the bucket is known) with a count per entry. Equal
// records meet in one entry; a record whose claim races with a writer may
// take a second entry, which only costs dedup, never a count. Once every
// record of the bucket is in the table, the distinct records overwrite the
// front of the bucket's own range (in place, no allocation) and their
// multiplicities go to cnt[] at the same indices; dlen[b] = their number. A
// bucket whose table fills keeps its records (dlen[b] = kRawList) and P5
// walks them with multiplicity 1.
// ---------------------------------------------------------------------------

constexpr int kRecProbe = 8;  // P5a: groups probed per record
#ifndef KC_P5A_PD
#define KC_P5A_PD 4
#endif
constexpr int kRecPd = KC_P5A_PD;  // P5a: record batches in flight per wave
#ifndef KC_P5A_BLOCK
#define KC_P5A_BLOCK 1024  // P5a workgroup
#endif
#ifndef KC_P5A_LDS
#define KC_P5A_LDS (160 * 1024)  // P5a LDS per workgroup (less: several workgroups per CU)
#endif
constexpr int kRecBlock = KC_P5A_BLOCK;
constexpr int kRecWaves = kRecBlock / 64;
static_assert(KC_P5A_LDS <= 160 * 1024 && (160 * 1024) / KC_P5A_LDS >= 1, "P5a LDS per workgroup: at most a CU's");
constexpr u32 kRecMaxSplit = 16;  // P5a: most hash-split passes of an overflowing bucket

struct RecDedupArgs {
    u64* recs;  // 2 x stride (SoA), grouped by bucket; distinct records written back in place
    u64 stride;
    const u64* starts;
    u32 b0, nbuckets;
    u32 ngrp;  // LDS groups of 2 entries
    u32* cnt;  // multiplicities, indexed like recs
    u32* dlen;
    // overflow lists: a bucket whose distinct records overflow the table is
    // deduplicated again in 2, 4, .. kRecMaxSplit passes, each taking the
    // records of one hash class, into a list reserved in the pool's free tail
    // [*over_cursor, over_limit) of recs (and cnt); dpos[b] = its start,
    // dlen[b] = kOverList | its length. over_cursor == nullptr: raw instead
    u64* over_cursor;
    u64 over_limit;
    u64* dpos;
};

__device__ __forceinline__ u32 rec_hash(u64 k0, u64 k1) {
    const u32 x = (u32)k0 ^ ((u32)(k0 >> 32) * 0x9e3779b1u);
    const u32 y = (u32)k1 ^ ((u32)(k1 >> 32) * 0x85ebca6bu);
    return fmix32(x ^ (y * 0xcc9e2d51u));
}

constexpr u32 kRecClaims = 4096;  // P5a: claimed entries listed for the write-back (u16 each)

static size_t rec_dedup_lds(u32 ngrp) { return (size_t)ngrp * 40 + 64 * 4 + 16 + kRecClaims * 2; }

u32 rec_dedup_groups() {
    u32 g = (u32)((KC_P5A_LDS - 64 * 4 - 16 - 64 - kRecClaims * 2) / 40);
    return g & ~15u;
}

// starts_r: a.starts as a read-only kernel argument, so a bucket's range is a
// scalar load that never waits behind the record loads and write-back stores
// in flight (in-order vmcnt)
__global__ __launch_bounds__(kRecBlock) void count_rec_k(RecDedupArgs a, const u64* __restrict__ starts_r) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64* tab = (u64*)smem;                        // entry e: tab[2e] = marked word 0, tab[2e + 1] = word 1
    u32* cnt = (u32*)(tab + 4 * (size_t)a.ngrp);  // 2 ngrp
    u32* misc = cnt + 2 * (size_t)a.ngrp;         // [0] overflow, [1..16] wave totals, [17] write-back cursor,
                                                  // [18] claims listed, [20..21] overflow list start (u64)
    unsigned short* clist = (unsigned short*)(misc + 64);  // entries in claim order (kRecClaims)
    const int tid = threadIdx.x, lane = (int)lane_id(), wave = tid >> 6;
    const u32 nent = 2 * a.ngrp;
    const u64 lt = lanemask_lt();
    for (u32 i = tid; i < nent; i += kRecBlock) {
        tab[2 * (size_t)i] = 0ull;
        tab[2 * (size_t)i + 1] = 0ull;
        cnt[i] = 0;
    }
    if (tid == 0) {
        misc[0] = 0;
        misc[17] = 0;
        misc[18] = 0;
    }
    __syncthreads();
    constexpr u64 kMark = 0x8000ull << 48;  // replaces the bucket bits: a non-zero word 0
    constexpr u64 kLow48 = (1ull << 48) - 1ull;
    // one record per lane, kRecPd batches in flight; a bucket's first batches
    // are loaded while the previous bucket is written out
    u64 n0[kRecPd], n1[kRecPd];
    auto share = [&](u32 bb, u64* wlo, u64* whi) {
        const u64 lo = starts_r[bb], hi = starts_r[bb + 1];
        const u64 nr = hi - lo, per_w = (nr + kRecWaves - 1) / kRecWaves;
        *wlo = lo + min(nr, (u64)wave * per_w);
        *whi = lo + min(nr, (u64)(wave + 1) * per_w);
    };
    auto prefetch = [&](u32 bb) {
        u64 wlo = 0, whi = 0;
        if (bb < a.nbuckets) share(bb, &wlo, &whi);
#pragma unroll
        for (int d = 0; d < kRecPd; d++) {
            const u64 i = wlo + (u64)d * 64 + lane;
            n0[d] = i < whi ? __builtin_nontemporal_load(a.recs + i) : 0ull;
            n1[d] = i < whi ? __builtin_nontemporal_load(a.recs + a.stride + i) : 0ull;
        }
    };
    // one record into the table (probing kRecProbe groups; a lost claim race
    // reads the group again): false when it found no place
    auto insert = [&](u64 k0, u64 k1, bool act, u32* claims) -> bool {
        u32 g = __umulhi(rec_hash(k0, k1), a.ngrp);
        bool done = !act;
        for (int pr = 0; pr < kRecProbe; pr++) {
            if (!__ballot(!done)) break;
            if (!done) {
                // (entry j of group g is entry 2g + (j ^ sw): the group's two
                // 16-byte entries swap places in every other run of 8 groups,
                // spreading a wave's loads over all 16 four-bank quads)
                const u32 sw = gswz(g) >> 1;
                const v2u64 e0 = *(const lds_v2u64*)(tab + 4 * (size_t)g + 2 * sw);
                const v2u64 e1 = *(const lds_v2u64*)(tab + 4 * (size_t)g + 2 * (sw ^ 1u));
                if (e0.x == k0 && e0.y == k1) {
                    atomicAdd(&cnt[2 * g + sw], 1u);
                    done = true;
                } else if (e1.x == k0 && e1.y == k1) {
                    atomicAdd(&cnt[2 * g + (sw ^ 1u)], 1u);
                    done = true;
                } else if (e0.x == 0ull || e1.x == 0ull) {
                    const u32 e = e0.x == 0ull ? 2 * g + sw : 2 * g + (sw ^ 1u);
                    const u64 old = atomicCAS((unsigned long long*)&tab[2 * (size_t)e], 0ull, (unsigned long long)k0);
                    if (old == 0ull) {
                        tab[2 * (size_t)e + 1] = k1;
                        atomicAdd(&cnt[e], 1u);
                        done = true;
                        ++*claims;
                        const u32 ci = atomicAdd(&misc[18], 1u);
                        if (ci < kRecClaims) clist[ci] = (unsigned short)e;
                    }
                    // lost the entry: the group is read again
                } else {
                    g = g + 1 == a.ngrp ? 0 : g + 1;
                }
            }
        }
        return done;
    };
    // the table's distinct records (the entries taken) to recs / cnt from
    // dst0 on, bucket bits b restored (put = false: only cleared); every
    // entry is cleared. Returns their number. Ends with the table and the
    // counters clear (two barriers inside).
    auto write_back = [&](u32 b, u64 dst0, u32 claims, bool put) -> u32 {
        for (int o2 = 32; o2 >= 1; o2 >>= 1) claims += (u32)__shfl_xor((int)claims, o2);
        if (lane == 0) misc[1 + wave] = claims;
        __syncthreads();
        u32 total = 0;
        for (int w = 0; w < kRecWaves; w++) total += misc[1 + w];
        if (total <= kRecClaims) {
            // the claimed entries in claim order: distinct record i goes to
            // dst0 + i, its entry is cleared
            for (u32 i = (u32)tid; i < total; i += kRecBlock) {
                const u32 e = clist[i];
                if (put) {
                    const u64 q = dst0 + i;
                    a.recs[q] = (tab[2 * (size_t)e] & kLow48) | ((u64)b << 48);
                    a.recs[a.stride + q] = tab[2 * (size_t)e + 1];
                    a.cnt[q] = cnt[e];
                }
                tab[2 * (size_t)e] = 0ull;
                tab[2 * (size_t)e + 1] = 0ull;
                cnt[e] = 0;
            }
        } else {
            const u32 spw = (nent + kRecWaves - 1) / kRecWaves;
            const u32 s0 = (u32)wave * spw, s1 = min(nent, s0 + spw);
            for (u32 c0 = s0; c0 < s1; c0 += 64) {
                const u32 i = c0 + (u32)lane;
                const bool occ = i < s1 && tab[2 * (size_t)i] != 0ull;
                const u64 bm = __ballot(occ);
                if (bm) {
                    u32 wb = 0;
                    if (lane == 0 && put) wb = atomicAdd(&misc[17], (u32)__popcll(bm));
                    wb = (u32)__builtin_amdgcn_readfirstlane((int)wb);
                    if (occ) {
                        if (put) {
                            const u64 q = dst0 + wb + (u64)__popcll(bm & lt);
                            a.recs[q] = (tab[2 * (size_t)i] & kLow48) | ((u64)b << 48);
                            a.recs[a.stride + q] = tab[2 * (size_t)i + 1];
                            a.cnt[q] = cnt[i];
                        }
                        tab[2 * (size_t)i] = 0ull;
                        tab[2 * (size_t)i + 1] = 0ull;
                        cnt[i] = 0;
                    }
                }
            }
        }
        __syncthreads();
        if (tid == 0) {
            misc[0] = 0;
            misc[17] = 0;
            misc[18] = 0;
        }
        __syncthreads();
        return total;
    };
    // buckets with more records than the table has entries: how many this
    // workgroup has seen and how many of them held too many distinct records
    // (uniform values); when most overflowed, such a bucket goes straight to
    // the hash-split passes instead of a first attempt that fills the table
    u32 big_seen = 0, big_over = 0;
    bool room = true;  // the overflow lists' space was not found exhausted
    prefetch(a.b0 + blockIdx.x);
    for (u32 b = a.b0 + blockIdx.x; b < a.nbuckets; b += gridDim.x) {
        u64 wlo, whi;
        share(b, &wlo, &whi);
        const u64 nrec_b = starts_r[b + 1] - starts_r[b];
        const bool big = nrec_b > (u64)nent;
        const bool skip_first = big && a.over_cursor && room && 2 * big_over > big_seen;
        bool over = false;
        u32 claims = 0;  // entries this lane took
        for (u64 base = wlo; base < whi && !skip_first; base += 64) {
            // a full table (any wave) ends the attempt: the bucket is split
            // or left raw, its remaining records are not needed now
            if (__hip_atomic_load(&misc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
            const bool act = base + lane < whi;
            const u64 k0 = (n0[0] & kLow48) | kMark, k1 = n1[0];
#pragma unroll
            for (int d = 0; d + 1 < kRecPd; d++) {
                n0[d] = n0[d + 1];
                n1[d] = n1[d + 1];
            }
            {
                const u64 i = base + (u64)kRecPd * 64 + lane;
                n0[kRecPd - 1] = i < whi ? __builtin_nontemporal_load(a.recs + i) : 0ull;
                n1[kRecPd - 1] = i < whi ? __builtin_nontemporal_load(a.recs + a.stride + i) : 0ull;
            }
            over |= !insert(k0, k1, act, &claims);
            if (__ballot(over) && lane == 0) atomicOr(&misc[0], 1u);
        }
        __syncthreads();
        // every record of the bucket is in the table: the next bucket's first
        // batches go in flight, then the distinct records are written back
        prefetch(b + gridDim.x);
        const bool raw = skip_first || misc[0] != 0u;
        const u64 pos0 = starts_r[b];
        if (!raw) {
            const u32 total = write_back(b, pos0, claims, true);
            if (tid == 0) a.dlen[b] = total;
            big_seen += big ? 1u : 0u;
            continue;
        }
        if (!skip_first) write_back(b, 0, claims, false);  // (clears the partial table)
        // overflow: the bucket's records again, in m passes by hash class,
        // into a list reserved in the pool's free tail (the bucket's own range
        // must stay intact for the later passes)
        const u64 nrec = starts_r[b + 1] - pos0;
        if (tid == 0) {
            u64 at = ~0ull;
            if (a.over_cursor) {
                at = atomicAdd((unsigned long long*)a.over_cursor, (unsigned long long)nrec);
                if (at + nrec > a.over_limit) at = ~0ull;  // no room: the bucket stays raw
            }
            *(u64*)(misc + 20) = at;
        }
        __syncthreads();
        const u64 lst = *(const u64*)(misc + 20);
        u32 m = 2, written = 0;
        bool ok = lst != ~0ull;
        room = room && ok;
        while (ok) {
            written = 0;
            bool again = false;
            for (u32 sub = 0; sub < m && !again; sub++) {
                bool ov = false;
                u32 cl = 0;
                // the wave's share again, the next batch's records in flight
                u64 p0 = wlo + lane < whi ? a.recs[wlo + lane] : 0ull;
                u64 p1 = wlo + lane < whi ? a.recs[a.stride + wlo + lane] : 0ull;
                for (u64 base = wlo; base < whi; base += 64) {
                    if (__hip_atomic_load(&misc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                    const bool in = base + lane < whi;
                    const u64 r0 = p0, r1 = p1;
                    const u64 i = base + 64 + lane;
                    p0 = i < whi ? a.recs[i] : 0ull;
                    p1 = i < whi ? a.recs[a.stride + i] : 0ull;
                    const u64 k0 = (r0 & kLow48) | kMark;
                    const bool act = in && (rec_hash(k0, r1) & (m - 1u)) == sub;
                    ov |= !insert(k0, r1, act, &cl);
                    if (__ballot(ov) && lane == 0) atomicOr(&misc[0], 1u);
                }
                __syncthreads();
                again = misc[0] != 0u;
                // (a pass that overflowed is cleared and the split doubles)
                written += write_back(b, lst + written, cl, !again);
            }
            if (!again) break;
            m *= 2;
            ok = m <= kRecMaxSplit;
        }
        if (tid == 0) {
            a.dlen[b] = ok ? (kOverList | written) : kRawList;
            if (ok) a.dpos[b] = lst;
        }
        if (big) {
            // (a skipped first attempt counts as an overflow only when the
            // bucket's distinct records would not have fit the table)
            big_seen++;
            big_over += (!skip_first || !ok || written > nent - nent / 8) ? 1u : 0u;
        }
    }
}

__global__ __launch_bounds__(kBlock) void dedup_total_k(const u32* __restrict__ dlen, const u64* __restrict__ starts,
                                                       u32 nb, u64* stats) {
    u64 v = 0;
    for (u32 b = blockIdx.x * kBlock + threadIdx.x; b < nb; b += gridDim.x * kBlock)
        v += dlen[b] == kRawList ? starts[b + 1] - starts[b] : (u64)(dlen[b] & ~kOverList);
    wave_add(&stats[ST_DEDUP], v);
}

hipError_t launch_dedup_total(const uint32_t* dlen, const uint64_t* starts, uint32_t nb, uint64_t* stats,
                              hipStream_t s) {
    hipLaunchKernelGGL(dedup_total_k, dim3(64), dim3(kBlock), 0, s, dlen, starts, nb, stats);
    return hipGetLastError();
}

hipError_t launch_count_rec(uint64_t* recs, uint64_t stride, const uint64_t* starts, uint32_t b0, uint32_t b1,
                            uint32_t* cnt, uint32_t* dlen, int grid, hipStream_t s, uint64_t* over_cursor,
                            uint64_t over_limit, uint64_t* dpos) {
    if (b1 <= b0) return hipSuccess;
    RecDedupArgs a;
    a.over_cursor = test_hook("KC_P5A_NO_SPLIT") ? nullptr : over_cursor;
    a.over_limit = over_limit;
    a.dpos = dpos;
    a.recs = recs;
    a.stride = stride;
    a.starts = starts;
    a.b0 = b0;
    a.nbuckets = b1;
    a.ngrp = rec_dedup_groups();
    if (const char* e = test_hook("KC_P5A_GROUPS")) {  // tests: force full tables (raw buckets)
        const long v = atol(e);
        if (v > 0 && (u32)v < a.ngrp) a.ngrp = (u32)v;
    }
    a.cnt = cnt;
    a.dlen = dlen;
    const size_t lds = (rec_dedup_lds(a.ngrp) + 15) & ~(size_t)15;
    // grid: n_cu workgroups per 160 KiB of LDS per workgroup
    hipLaunchKernelGGL(count_rec_k, dim3(grid * ((160 * 1024) / KC_P5A_LDS)), dim3(kRecBlock), lds, s, a, a.starts);
    return hipGetLastError();
}

int seg_sort_cap(int W) {
    switch (W) {
    case 1: return SegCfg<1>::CAP;
    case 2: return SegCfg<2>::CAP;
    case 3: return SegCfg<3>::CAP;
    default: return SegCfg<4>::CAP;
    }
}
