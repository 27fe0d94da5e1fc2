// kc_synth.h — synthetic FASTQ generator shared by the host writer and the
// device kernel (bench/test input only; never on the counting path).
//
// Record i: "@r<i>\n" <seq: L bases> "\n+\n" <'I' x L> "\n".
// Bases come from splitmix64 draws keyed by (seed, stream, index), so any
// record can be produced independently: reads shard by index and the host and
// device generators emit identical bytes (tests/test_gpu_parity.py checks it).
//   genome mode (genome_length G > 0): read i starts at
//       pos_i = rand(seed, 1, i) mod (G - L + 1)
//     and base j is genome base g = pos_i + j, taken from word rand(seed, 2, g/32),
//     bits 2*(g%32)..+1 -> "ACGT".
//   iid mode (G == 0): base j of read i is bits 2*(j%32) of
//       rand(seed, 4, i*ceil(L/32) + j/32).
//   N replacement: base j of read i becomes 'N' when
//       (rand(seed, 3, i*L + j) >> 11) < n_threshold,  n_threshold = n_rate * 2^53.
//   Variable read lengths (Lmin in [1, L)): read i keeps its first
//       len_i = Lmin + rand(seed, 5, i) mod (L - Lmin + 1) bases (sequence and
//       quality lines), and its header gains 2 (L - len_i) 'x' bytes, so every
//       record keeps the fixed-length record's size and offset.
//   Layout 1 (chunks): only the sequences, read i at (i - first) * L — the
//       bytes FASTQFileReader::readData concatenates into a reference chunk
//       (FASTQFileReader.cpp:49-89); fixed read length only.
#pragma once
#include <stdint.h>

#define KC_SYNTH_HD __host__ __device__ inline

KC_SYNTH_HD uint64_t kc_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

KC_SYNTH_HD uint64_t kc_synth_rand(uint64_t seed, uint64_t stream, uint64_t i) {
    return kc_splitmix64(kc_splitmix64(seed ^ (stream * 0xD1342543DE82EF95ull)) + i);
}

KC_SYNTH_HD uint32_t kc_synth_digits(uint64_t i) {
    uint32_t d = 1;
    while (i >= 10) {
        i /= 10;
        d++;
    }
    return d;
}

// Sum of decimal digit counts of 0 .. x-1.
KC_SYNTH_HD uint64_t kc_synth_digit_sum(uint64_t x) {
    uint64_t total = 0, lo = 0, hi = 10;
    uint32_t d = 1;
    while (x > lo) {
        uint64_t top = x < hi ? x : hi;
        total += (top - lo) * d;
        if (hi > 1000000000000000000ull) break;
        lo = hi;
        hi *= 10;
        d++;
    }
    return total;
}

// Byte offset of record i inside a buffer that starts with record `first`.
KC_SYNTH_HD uint64_t kc_synth_offset(uint64_t first, uint64_t i, int64_t L) {
    return (i - first) * (uint64_t)(2 * L + 7) + kc_synth_digit_sum(i) - kc_synth_digit_sum(first);
}

struct kc_synth_params {
    uint64_t first, n, seed, genome, n_threshold;
    int64_t L;
    int64_t Lmin;  // 0: every read has L bases
    int layout;    // 0: FASTQ records, 1: concatenated sequences (reference chunk layout)
};

KC_SYNTH_HD int64_t kc_synth_len(const kc_synth_params& p, uint64_t i) {
    if (p.Lmin <= 0 || p.Lmin >= p.L) return p.L;
    return p.Lmin + (int64_t)(kc_synth_rand(p.seed, 5, i) % (uint64_t)(p.L - p.Lmin + 1));
}

KC_SYNTH_HD char kc_synth_base(const kc_synth_params& p, uint64_t i, int64_t j, uint64_t pos) {
    uint32_t c;
    if (p.genome > 0) {
        uint64_t g = pos + (uint64_t)j;
        c = (uint32_t)(kc_synth_rand(p.seed, 2, g >> 5) >> (2 * (g & 31))) & 3u;
    } else {
        uint64_t wpr = (uint64_t)((p.L + 31) / 32);
        c = (uint32_t)(kc_synth_rand(p.seed, 4, i * wpr + (uint64_t)(j >> 5)) >> (2 * (j & 31))) & 3u;
    }
    if (p.n_threshold && (kc_synth_rand(p.seed, 3, i * (uint64_t)p.L + (uint64_t)j) >> 11) < p.n_threshold) return 'N';
    return "ACGT"[c];
}

// Writes the L bases of read i at dst (layout 1).
KC_SYNTH_HD void kc_synth_sequence(const kc_synth_params& p, uint64_t i, char* dst) {
    uint64_t pos = 0;
    if (p.genome > 0) pos = kc_synth_rand(p.seed, 1, i) % (p.genome - (uint64_t)p.L + 1);
    for (int64_t j = 0; j < p.L; j++) dst[j] = kc_synth_base(p, i, j, pos);
}

// Writes record i at dst (which points at the record's first byte).
KC_SYNTH_HD void kc_synth_record(const kc_synth_params& p, uint64_t i, char* dst) {
    char digits[24];
    uint32_t nd = 0;
    uint64_t v = i;
    do {
        digits[nd++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    char* o = dst;
    *o++ = '@';
    *o++ = 'r';
    while (nd) *o++ = digits[--nd];
    const int64_t len = kc_synth_len(p, i);
    for (int64_t j = 0; j < 2 * (p.L - len); j++) *o++ = 'x';
    *o++ = '\n';
    uint64_t pos = 0;
    if (p.genome > 0) pos = kc_synth_rand(p.seed, 1, i) % (p.genome - (uint64_t)p.L + 1);
    for (int64_t j = 0; j < len; j++) *o++ = kc_synth_base(p, i, j, pos);
    *o++ = '\n';
    *o++ = '+';
    *o++ = '\n';
    for (int64_t j = 0; j < len; j++) *o++ = 'I';
    *o++ = '\n';
}
