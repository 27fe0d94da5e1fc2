// rp_bench: the radix scatter (rp_scatter_k, S / P3 / P3b) alone on random
// records, timed with HIP events; run against variant builds of
// libkc_hip.so (tools/build_variant.sh, KC_RP_ABL ablations) through
// LD_LIBRARY_PATH. Usage: rp_bench [n_records] [NW] [reps] [emit] [dshift] [layout]
// Every run checks its output (digits ascending, items' hash sum equal to the
// input's, emitted digit bytes).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "kc_device.h"

// RP_PAD experiment: digit d's output run starts d x pad records later (gaps
// between the 256 digit regions; the output check is skipped then)
__global__ void pad_pos_k(uint64_t* pos, uint64_t n, uint64_t pad) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        pos[i] += (i & 255) * pad;
}

__global__ void fill_k(uint64_t* a, uint64_t n, int NW, uint64_t seed) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        for (int j = 0; j < NW; j++) {
            uint64_t x = (i + 1) * 0x9e3779b97f4a7c15ull + seed + (uint64_t)j * 0x632be59bd9b4e019ull;
            x ^= x >> 31;
            x *= 0xbf58476d1ce4e5b9ull;
            x ^= x >> 29;
            a[(uint64_t)j * n + i] = x;
        }
    }
}

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 592344064ull;
    const int NW = argc > 2 ? atoi(argv[2]) : 2;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const bool with_emit = argc > 4 ? atoi(argv[4]) != 0 : true;  // digit bytes for the next level
    const int dshift = argc > 5 ? atoi(argv[5]) : 48;  // 56 + 6 = 62: 4 digits, long runs
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    const uint64_t tile = (uint64_t)kc::rp_tile(NW, false);
    const uint64_t nt = (n + tile - 1) / tile;
    uint64_t *a, *b, *rt, *pos, *tmp;
    uint8_t* digs;
    // layout -1: two allocations; -2: two physically contiguous ones; -3: two
    // of three regions each, six (input, output) region pairs timed in one
    // process; >= 0: one, b at a + its size + layout bytes
    const long long layout = argc > 6 ? atoll(argv[6]) : -1;
    // -3: RP_NREG (default 3) regions per buffer, (input, output) pairs timed in one process
    const int nreg = layout == -3 ? (getenv("RP_NREG") ? atoi(getenv("RP_NREG")) : 3) : 1;
    uint64_t padn = 0;
    for (const char* q = getenv("RP_PADS") ? getenv("RP_PADS") : getenv("RP_PAD"); q && *q;) {
        const uint64_t v = 256 * strtoull(q, nullptr, 10);
        if (v > padn) padn = v;
        const char* c = strchr(q, ',');
        q = c ? c + 1 : nullptr;
    }
    const uint64_t ob = n + padn;  // output stride (records)
    // -4: the output in three places, timed as pairs (0, r): r = 0 a plain
    // allocation, 1 mapped from RP_CHUNK_MB physical chunks in creation order
    // (virtual memory API), 2 the same chunks mapped in a shuffled order
    std::vector<uint64_t*> outs;
    if (layout == -4) {
        CK(hipMalloc(&a, n * 8 * NW));
        uint64_t* p0;
        CK(hipMalloc(&p0, ob * 8 * NW));
        outs.push_back(p0);
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = 0;
        size_t gran = 0;
        CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
        const size_t chunk = std::max<size_t>(gran, (size_t)(getenv("RP_CHUNK_MB") ? atoi(getenv("RP_CHUNK_MB")) : 64) << 20);
        const size_t bytes = ((ob * 8 * NW + chunk - 1) / chunk) * chunk;
        const size_t nch = bytes / chunk;
        fprintf(stderr, "rp_bench: granularity %zu, chunk %zu, %zu chunks per mapped buffer\n", gran, chunk, nch);
        for (int v = 0; v < 2; v++) {
            void* va = nullptr;
            CK(hipMemAddressReserve(&va, bytes, 0, nullptr, 0));
            std::vector<hipMemGenericAllocationHandle_t> hs(nch);
            for (size_t i = 0; i < nch; i++) CK(hipMemCreate(&hs[i], chunk, &prop, 0));
            std::vector<size_t> perm(nch);
            for (size_t i = 0; i < nch; i++) perm[i] = i;
            if (v == 1) {
                uint64_t x = 88172645463325252ull;
                for (size_t i = nch - 1; i > 0; i--) {
                    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                    std::swap(perm[i], perm[x % (i + 1)]);
                }
            }
            for (size_t i = 0; i < nch; i++) CK(hipMemMap((char*)va + i * chunk, chunk, 0, hs[perm[i]], 0));
            hipMemAccessDesc acc = {};
            acc.location = prop.location;
            acc.flags = hipMemAccessFlagsProtReadWrite;
            CK(hipMemSetAccess(va, bytes, &acc, 1));
            outs.push_back((uint64_t*)va);
        }
        b = outs[0];
    } else if (layout == -3) {
        CK(hipMalloc(&a, nreg * n * 8 * NW));
        CK(hipMalloc(&b, nreg * ob * 8 * NW));
    } else if (layout == -2) {  // physically contiguous allocations
        CK(hipExtMallocWithFlags((void**)&a, n * 8 * NW, hipDeviceMallocContiguous));
        CK(hipExtMallocWithFlags((void**)&b, n * 8 * NW, hipDeviceMallocContiguous));
    } else if (layout < 0) {
        CK(hipMalloc(&a, n * 8 * NW));
        CK(hipMalloc(&b, ob * 8 * NW));
    } else {
        CK(hipMalloc(&a, 2 * n * 8 * NW + (uint64_t)layout + 256));
        b = (uint64_t*)((char*)a + ((n * 8 * NW + (uint64_t)layout + 255) & ~255ull));
    }
    CK(hipMalloc(&digs, ob + 64));
    CK(hipMalloc(&rt, 64));
    CK(hipMalloc(&pos, nt * 256 * 8));
    CK(hipMalloc(&tmp, nt * 256 * 8 + (64 << 20)));
    uint64_t h[4] = {0, n, 0, nt};
    CK(hipMemcpy(rt, h, 32, hipMemcpyHostToDevice));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int g = 0; g < nreg; g++)
        hipLaunchKernelGGL(fill_k, dim3(8192), dim3(256), 0, s, a + (uint64_t)g * n * NW, n, NW, 12345ull);
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // RP_PADS=p0,p1,...: the pairs are timed once per pad (the largest sizes
    // the output buffer; RP_PAD: one pad)
    std::vector<uint64_t> pads;
    {
        const char* e = getenv("RP_PADS") ? getenv("RP_PADS") : getenv("RP_PAD");
        for (const char* q = e; q && *q;) {
            pads.push_back(strtoull(q, nullptr, 10));
            const char* c = strchr(q, ',');
            q = c ? c + 1 : nullptr;
        }
        if (pads.empty()) pads.push_back(0);
    }
    for (uint64_t pad : pads) {
    CK(kc::launch_rp_hist(nullptr, a, dshift, rt, rt + 2, 1, nt, (uint32_t)tile, pos, tmp, 2 * ncu, s));
    if (pad) hipLaunchKernelGGL(pad_pos_k, dim3(1024), dim3(256), 0, s, pos, nt * 256, pad);
    const int R1 = nreg - 1, RH = nreg / 2;
    int pairs[64][2] = {{0, 0}, {0, nreg > 3 ? R1 : 1}, {nreg > 3 ? RH : 1, 0}, {nreg > 3 ? RH : 1, nreg > 3 ? RH : 1},
                        {R1, R1}, {R1, 0}};
    int npairs = 6;
    if (const char* e = getenv("RP_PAIRS")) {  // "i:o,i:o,..."
        npairs = 0;
        for (const char* q = e; q && *q && npairs < 64;) {
            pairs[npairs][0] = atoi(q);
            const char* c = strchr(q, ':');
            pairs[npairs][1] = c ? atoi(c + 1) : 0;
            npairs++;
            c = strchr(q, ',');
            q = c ? c + 1 : nullptr;
        }
    }
    const int sweeps = getenv("RP_SWEEPS") ? atoi(getenv("RP_SWEEPS")) : 1;  // repeat the pairs: stable?
    if (layout == -4 && !getenv("RP_PAIRS")) {
        npairs = 3;
        for (int r = 0; r < 3; r++) pairs[r][0] = 0, pairs[r][1] = r;
    }
    for (int pk = 0; pk < ((nreg > 1 || layout == -4) ? npairs * sweeps : 1); pk++) {
    const int pi = pk % npairs;
    uint64_t* ai = a + (layout == -4 ? 0 : (uint64_t)pairs[pi][0] * n * NW);
    uint64_t* bi = layout == -4 ? outs[pairs[pi][1]] : b + (uint64_t)pairs[pi][1] * ob * NW;
    float best = 1e30f, tot = 0.f;
    for (int r = 0; r < reps + 1; r++) {
        CK(hipEventRecord(e0, s));
        CK(kc::launch_rp_scatter(NW, false, ai, n, bi, ob, nullptr, nullptr, rt, rt + 2, 1, nt, pos, dshift,
                                 with_emit ? digs : nullptr, 56, 2 * ncu, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        if (r > 0) {
            tot += t;
            if (t < best) best = t;
        }
    }
    // check: output digits ascending, every item once (hash sums), emitted digit bytes
    if (!pad && !getenv("RP_NOCHECK")) {
        std::vector<uint64_t> hi((size_t)n * NW), ho((size_t)n * NW);
        std::vector<uint8_t> hd(with_emit ? n : 1);
        CK(hipMemcpy(hi.data(), ai, n * 8 * NW, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ho.data(), bi, n * 8 * NW, hipMemcpyDeviceToHost));
        if (with_emit) CK(hipMemcpy(hd.data(), digs, n, hipMemcpyDeviceToHost));
        uint64_t si = 0, so = 0, bad = 0;
        auto mix = [](uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; return x; };
        for (uint64_t i = 0; i < n; i++) {
            uint64_t x = 0, y = 0;
            for (int j = 0; j < NW; j++) {
                x = mix(x ^ hi[(size_t)j * n + i]) + (uint64_t)j;
                y = mix(y ^ ho[(size_t)j * n + i]) + (uint64_t)j;
            }
            si += x;
            so += y;
            if (i && ((ho[i] >> dshift) & 255) < ((ho[i - 1] >> dshift) & 255)) bad++;
            if (with_emit && hd[i] != (uint8_t)(ho[i] >> 56)) bad++;
        }
        if (si != so || bad) {
            fprintf(stderr, "rp_bench: output check FAILED (hash %s, %llu misplaced)\n", si == so ? "ok" : "differs",
                    (unsigned long long)bad);
            return 2;
        }
    }
    const double bytes = (double)n * (16.0 * NW + (with_emit ? 1.0 : 0.0));
    printf("{\"pad\": %llu, \"pair\": [%d, %d], \"dshift\": %d, \"n\": %llu, \"NW\": %d, \"emit\": %d, \"tile\": %llu, \"avg_ms\": %.3f, \"best_ms\": %.3f, \"GBps_avg\": %.1f}\n",
           (unsigned long long)pad, pairs[pi][0], pairs[pi][1], dshift, (unsigned long long)n, NW, with_emit ? 1 : 0, (unsigned long long)tile, tot / reps, best,
           bytes / (tot / reps / 1e3) / 1e9);
    }
    }
    return 0;
}
