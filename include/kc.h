/*
 * kc.h — C ABI of the MI355X-native k-mer counting path (libkc_hip.so).
 *
 * This is the drop-in boundary for the reference's device path. The reference
 * binds exactly three functions from its CUDA translation unit
 * (GPUHandler.h:61-65), all called from KMerCounter.cpp only:
 *
 *   GPUStream** PrepareGPU(uint32_t streamCount, uint64_t inputSize,
 *                          uint64_t lineLength, int64_t kmerLength);      GPUHandler.h:61
 *   int64_t     processKMers(GPUStream*, const char* input, int64_t kmerLength,
 *                            int64_t inputSize, int64_t lineLength,
 *                            uint32_t readId, FileDump&);                  GPUHandler.h:64
 *   void        FreeGPU(GPUStream**, uint32_t streamCount);               GPUHandler.h:62
 *
 * and then aggregates the returned records on the host in a TBB
 * concurrent_hash_map (KMerCounter.cpp:61-82) which it dumps at the end
 * (KMerCounter.cpp:91-106). Here the aggregation lives on the GPU (an
 * open-addressed table in HBM), so one context replaces a GPUStream pool plus
 * the host hash:
 *
 *   kc_create             replaces PrepareGPU            (GPUHandler.cu:479-509)
 *   kc_count_chunk        replaces processKMers + the host hash insert of
 *                         dispatchWork                   (GPUHandler.cu:397-477,
 *                                                         KMerCounter.cpp:51-89)
 *   kc_count_fastq        new: raw record-aligned FASTQ block, decoded on the GPU
 *                         (replaces FASTQFileReader::readData's host concatenation,
 *                         FASTQFileReader.cpp:49-89, for well-formed 4-line FASTQ)
 *   kc_finish/kc_write_output
 *                         replace DumpResults            (KMerCounter.cpp:91-106)
 *                         and the disabled sorted-spill merge
 *                         (KMerFileMergeHandler.cpp:49-100) — output is always
 *                         the SortedKMerFile format (SortedKMerFile.cpp:18-124).
 *   kc_destroy            replaces FreeGPU               (GPUHandler.cu:511-519)
 *
 * Error handling: the reference calls exit() on any CUDA error
 * (GPUHandler.h:27-34). Every entry point here returns a kc_status instead;
 * kc_last_error() gives a human-readable message for the last failure on a ctx.
 *
 * Threading: a ctx is bound to one HIP device and one HIP stream and is NOT
 * thread-safe; distinct ctxs (e.g. one per GPU) may be driven concurrently
 * from separate host threads (the reference drives 8 GPUStreams from 8
 * threads, KMerCounter.cpp:123-139).
 *
 * Record format of every output (SortedKMerFile): no header;
 * records of W = ceil(k/32) little-endian uint64 key words followed by a
 * little-endian uint32 count; rs = 8W+4 bytes; strictly ascending by the key
 * words compared as unsigned integers, word 0 first (KMerFileMerger.cpp:98-108).
 */
#ifndef KC_H
#define KC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KC_ABI_VERSION 7 /* 2: kc_stats.dedup_ms / dedup_records; 3: kc_synth_spec.min_read_length;
                            4: kc_count_file, kc_checkpoint / kc_rollback / kc_commit;
                            5: kc_stats.presplit_ms / presplit_batches / sorted_run_batches;
                            6: kc_stats.key_passes;
                            7: kc_stats.finish_group_ms, kc_merge_part_* */
#define KC_MAX_K 128 /* keys up to 4 words, the widest KMerSizes.h type (KMer128) */

typedef enum kc_status {
    KC_OK = 0,
    KC_ERR_ARG = 1,      /* invalid argument: k outside [1,128], L < k, L > 32767, ... */
    KC_ERR_HIP = 2,      /* a HIP runtime call failed (reference: gpuAssert -> exit) */
    KC_ERR_NOMEM = 3,    /* device or host allocation failed */
    KC_ERR_FORMAT = 4,   /* FASTQ block is not 4-line records with L-byte sequences */
    KC_ERR_IO = 5,       /* file open/read/write failed */
    KC_ERR_STATE = 6,    /* call not valid in the ctx's current state */
    KC_ERR_NODEVICE = 7, /* no HIP device / invalid device ordinal */
    KC_ERR_INTERNAL = 8  /* device-side invariant violated (bug) */
} kc_status;

typedef struct kc_ctx kc_ctx;

typedef struct kc_config {
    int32_t device;            /* HIP device ordinal */
    int32_t reserved0;
    int64_t kmer_length;       /* k: Options::GetKmerLength (Options.h:31) */
    int64_t line_length;       /* L: read length (FASTQFileReader.cpp:35) */
    uint64_t gpu_memory_limit; /* device working-set cap in bytes: hash table +
                                  spill buffer + staging (Options::GetGpuMemoryLimit,
                                  main.cpp:28 default 1e8). 0 = 1e8. */
    uint64_t table_bytes;      /* optional explicit hash-table size; 0 = derive
                                  from gpu_memory_limit */
    const char* temp_dir;      /* spill runs are written here as SortedKMerFile
                                  files (Options::getTempFileLocation); NULL or ""
                                  keeps spill runs in host memory */
    uint32_t flags;            /* KC_FLAG_* */
    uint32_t lds_slots;        /* partition engine: LDS table slots per bucket
                                  (0 = the maximum that fits; small values force
                                  the overflow path, for tests) */
} kc_config;

#define KC_FLAG_NONE 0u
#define KC_FLAG_QUIET 1u        /* no progress lines on stderr */
#define KC_FLAG_ENGINE_TABLE 2u  /* count with the global atomic hash table only */
#define KC_FLAG_ENGINE_SKM 4u    /* super-k-mer engine without the cardinality
                                    check (see below) */
#define KC_FLAG_ENGINE_PREFIX 8u /* key-prefix partition engine only: hash-free
                                    65536 buckets by the first 8 bases, each
                                    counted in an LDS table; sorted output needs
                                    no global sort */
#define KC_FLAG_VARLEN 16u      /* variable-length reads (an
                                    extension: the reference concatenates reads
                                    without separators and cuts at multiples of
                                    the first read's length, FASTQFileReader.cpp:
                                    57-79, so it has no defined result for them).
                                    kc_count_fastq* then accept 4-line records
                                    whose sequence lines hold 0..line_length
                                    bytes; every read counts the windows of a
                                    reference read of its own length (a read
                                    shorter than k counts none), and key 0^W is
                                    present iff a read of >= k bases holds a
                                    not-ACGT base or a key-0 window was counted.
                                    kc_stats.windows sums the reads' own
                                    windows. Not with KC_FLAG_ENGINE_TABLE
                                    (kc_create returns KC_ERR_ARG). */
/* Default engine (no ENGINE flag): the super-k-mer engine. Runs of consecutive
 * windows that share a minimizer bucket move through HBM as one record of
 * bases (~1.5 B per k-mer at k=31 instead of an 8-byte key), are grouped by
 * bucket and counted per bucket in an LDS table. Before counting a large
 * batch it counts a sample of buckets; when most sampled keys are distinct
 * (no coverage, e.g. iid reads) the key-prefix engine counts the batch and the
 * rest of the context's input instead. (L, k) outside its range (k < 18,
 * k > 96, reads > 4096 + k - 1 bases) use the key-prefix engine. Every engine
 * gives the same bytes. */

typedef struct kc_stats {
    uint64_t reads;            /* reads counted so far */
    uint64_t windows;          /* k-mer windows examined: reads * (L-k+1) */
    uint64_t valid_kmers;      /* windows without an invalid base (= sum of counts) */
    uint64_t table_capacity;   /* slots */
    uint64_t table_used;       /* occupied slots after kc_finish */
    uint64_t spilled_kmers;    /* k-mers routed to the spill path */
    uint64_t spill_runs;       /* sorted spill runs produced */
    uint64_t output_records;   /* distinct keys in the final output */
    uint64_t insert_launches;  /* count_kmers kernel launches since the last reset */
    double insert_ms;          /* summed device time of those launches (HIP events) */
    double decode_ms;          /* FASTQ index + validate kernels */
    double finish_ms;          /* kc_finish's device time: compact + group/sort + pack */
    double last_count_ms;      /* device time of the last kc_count_* call */
    double part_ms[5];         /* partition engine (summed device time): [0] encode
                                  (E) + P1 digit histogram, [1] P2 scatter,
                                  [2] P3 regional scatter kernel, [3] P3 tile
                                  histograms + scan + P4 bucket bounds, [4] P5
                                  LDS bucket count */
    uint64_t batches;          /* partition engine batches */
    uint64_t keys;             /* partition engine: keys partitioned (valid,
                                  non-zero windows) since the last reset */
    uint64_t p5_launches;      /* P5 launches (reruns on record overflow included) */
    uint32_t engines_used;     /* bit 0: super-k-mer, bit 1: key-prefix partition,
                                  bit 2: global table (batches since the last reset) */
    uint32_t reserved1;
    double dedup_ms;           /* super-k-mer engine, W = 1: summed device time of
                                  P5a (identical records of a bucket counted once);
                                  part_ms[4] is then the weighted P5 walk alone */
    uint64_t dedup_records;    /* distinct records P5a listed since the last reset */
    double presplit_ms;        /* key-prefix engine, high cardinality: summed device
                                  time of P3b (every bucket split by key bits 40..47:
                                  histogram, scatter, sub-bucket starts); included in
                                  part_ms[2] */
    uint64_t presplit_batches; /* batches that took P3b */
    uint64_t sorted_run_batches; /* batches counted by P5s (runs of sub-buckets sorted
                                    in LDS; part_ms[4] holds their time) */
    uint64_t key_passes;       /* key-prefix engine, high cardinality: key-range passes
                                  (a batch too big for the working set counted by
                                  disjoint key ranges whose runs concatenate) */
    double finish_group_ms;    /* part of finish_ms: the super-k-mer finish's two
                                  grouping passes (histograms + radix scatters of the
                                  (key, count) records by their first 8 bases) */
} kc_stats;

/* Synthetic FASTQ. Records are "@r<i>\n<seq>\n+\n<'I' x L>\n". (ABI 4: layout) */
typedef struct kc_synth_spec {
    uint64_t n_reads;
    int64_t read_length;   /* L */
    uint64_t seed;
    uint64_t genome_length;/* 0 = iid uniform bases; >0 = reads sampled from a
                              random genome of this many bases */
    double n_rate;         /* probability that a base is replaced by 'N' */
    uint64_t first_read;   /* index of the first record to emit (for sharding) */
    int64_t min_read_length; /* 0 = every read has read_length bases; in
                              [1, read_length): read i keeps its first
                              min + rand(i) mod (read_length - min + 1) bases
                              and its header is padded with 'x' to keep the
                              record size (variable-length input, KC_FLAG_VARLEN) */
    uint32_t layout;       /* 0 = FASTQ records; 1 = the sequences only, read i at
                              (i - first_read) * read_length: the bytes of a
                              reference chunk (FASTQFileReader.cpp:49-89), for
                              kc_count_chunk (fixed read length only) */
    uint32_t reserved;
} kc_synth_spec;

/* ---- lifecycle ---------------------------------------------------------- */
kc_status kc_create(kc_ctx** out, const kc_config* cfg);
void kc_destroy(kc_ctx* ctx);
const char* kc_strerror(kc_status s);
const char* kc_last_error(const kc_ctx* ctx);
int32_t kc_abi_version(void);
/* Number of visible HIP devices (0 when none; never fails). */
int32_t kc_device_count(void);
/* Forget every count (table, spill runs, stats); keeps allocations. */
kc_status kc_reset(kc_ctx* ctx);

/* ---- counting ----------------------------------------------------------- */
/* Reference-exact chunk: `size` bytes of concatenated L-byte sequences, exactly
 * what FASTQFileReader::readData hands to processKMers. floor(size/L) reads are
 * counted; a trailing partial read is ignored (GPUHandler.cu:13-15). `chunk` is
 * a host pointer owned by the caller and may be reused when the call returns. */
kc_status kc_count_chunk(kc_ctx* ctx, const char* chunk, int64_t size, int64_t line_length);
/* Same, `d_chunk` is device memory on the ctx's device. */
kc_status kc_count_chunk_device(kc_ctx* ctx, const void* d_chunk, int64_t size, int64_t line_length);
/* Record-aligned block of raw FASTQ text (host memory). Must consist of whole
 * 4-line records whose sequence line is exactly `line_length` bytes (0 = the
 * ctx's configured L) and end with '\n'; otherwise returns KC_ERR_FORMAT
 * without counting anything from the block. *n_reads (may be NULL) receives
 * the number of records in the block. The sequence lines are exactly the lines
 * FASTQFileReader::readData concatenates (the line before each '+' line). */
kc_status kc_count_fastq(kc_ctx* ctx, const char* fastq, uint64_t n_bytes, int64_t line_length, uint64_t* n_reads);
/* Same, `d_fastq` is device memory on the ctx's device. */
kc_status kc_count_fastq_device(kc_ctx* ctx, const void* d_fastq, uint64_t n_bytes, int64_t line_length,
                                uint64_t* n_reads);
/* Validation only (the GPU index of kc_count_fastq without counting). */
kc_status kc_check_fastq(kc_ctx* ctx, const char* fastq, uint64_t n_bytes, int64_t line_length, uint64_t* n_reads);

/* Batching. kc_count_chunk / kc_count_fastq* decode and 2-bit encode each
 * block on the GPU at once (a malformed FASTQ block is reported by its own
 * call) but count the encoded reads in batches: a batch is counted when the
 * next block does not fit it (gpu_memory_limit), when the read length
 * changes, or at kc_finish. Many small calls (the reference's 7.8 MB chunks)
 * therefore cost about what one large block costs. Host buffers may be reused
 * as soon as a call returns. */

/* Checkpoint of the ctx's input: kc_rollback forgets every block counted
 * since, as long as no batch was counted in between (KC_ERR_STATE otherwise;
 * while a checkpoint is held, batches grow up to 1/8 of device memory before
 * they are counted). kc_commit drops the checkpoint. Used by kc_count_file's
 * auto mode to fall back to the reference chunker after a malformed block
 * without reading the file twice. */
kc_status kc_checkpoint(kc_ctx* ctx);
kc_status kc_rollback(kc_ctx* ctx);
kc_status kc_commit(kc_ctx* ctx);

/* Whole FASTQ file (replaces InputFileHandler::read + FASTQFileReader::readData,
 * InputFileHandler.cpp:82-95, FASTQFileReader.cpp:49-89, and the chunk loop of
 * KMerCounter::Start, KMerCounter.cpp:123-143). The file is read in 256 MiB
 * blocks (pread into pinned buffers, read ahead of the GPU), cut at record
 * boundaries, and each block goes to one of the n_ctx contexts (read-shard: a
 * block to whichever context is free). line_length 0 = the file's line 2
 * (FASTQFileReader.cpp:31-35; the ctx's L with KC_FLAG_VARLEN); a file whose
 * reads are shorter than k counts nothing. mode:
 *   KC_INPUT_AUTO  : GPU FASTQ decode; if a block is not 4-line records of
 *                    L-base reads, the whole file is counted in the
 *                    reference's own chunks instead (as KC_INPUT_EXACT) —
 *                    bit-exact with the reference on any input;
 *   KC_INPUT_FASTQ : GPU FASTQ decode; a malformed block is KC_ERR_FORMAT;
 *   KC_INPUT_EXACT : the reference's chunker (readData with the chunk size of
 *                    KMerCounter::GetChunkSize from gpu_memory_limit, header
 *                    >= 2L records lost at chunk edges as in the reference)
 *                    on ctxs[0], through kc_count_chunk.
 * Variable-length contexts always decode FASTQ. *n_reads (may be NULL)
 * receives the reads counted. */
#define KC_INPUT_AUTO 0u
#define KC_INPUT_FASTQ 1u
#define KC_INPUT_EXACT 2u
kc_status kc_count_file(kc_ctx* const* ctxs, uint32_t n_ctx, const char* path, int64_t line_length, uint32_t mode,
                        uint64_t* n_reads);

/* ---- results ------------------------------------------------------------ */
/* Compacts and radix-sorts the hash table on the device. *n_records receives
 * the number of records of the table run (spill runs not included). After
 * kc_finish no more counting is allowed until kc_reset. */
kc_status kc_finish(kc_ctx* ctx, uint64_t* n_records);
/* Copies the sorted table run as SortedKMerFile bytes (n_records * rs) to host
 * memory. Valid only when no spill run exists (see kc_stats.spill_runs). */
kc_status kc_copy_records(kc_ctx* ctx, void* dst, uint64_t dst_bytes);
/* Device pointer + byte size of the sorted table run as SortedKMerFile bytes
 * (valid until kc_reset/kc_destroy). */
kc_status kc_device_records(kc_ctx* ctx, const void** d_records, uint64_t* n_bytes);
/* Writes the final SortedKMerFile: the table run k-way merged with every spill
 * run (KMerFileMergeHandler semantics: groups of `merge_fan_in` files merged by
 * up to `merge_threads` threads, equal keys summed as uint32). The file is
 * truncated first (the reference appends, KMerFileMerger.cpp:129). */
kc_status kc_write_output(kc_ctx* ctx, const char* path, uint32_t merge_fan_in, uint32_t merge_threads);
/* Writes the finished table run (no spill runs) into an existing file at byte
 * `offset` without truncating it: the ranks of a key-space exchange write
 * their key ranges of one output file side by side. */
kc_status kc_write_output_at(kc_ctx* ctx, const char* path, uint64_t offset);
/* Writes the table run plus spill runs as separate sorted run files
 * "<prefix>.<i>" and returns how many were written (for multi-GPU merges). */
kc_status kc_write_runs(kc_ctx* ctx, const char* prefix, uint32_t* n_runs);
kc_status kc_get_stats(const kc_ctx* ctx, kc_stats* out);

/* ---- key-space partition across GPUs ----------------------
 * owner(key) = ((word0 >> 32) * world) >> 32 is monotone in the key, so after
 * every rank sends owner o the records of its sorted table run that o owns and
 * o merges what it receives, the ranks' outputs concatenated in rank order
 * are the global SortedKMerFile. The exchange itself is the caller's
 * (an RCCL all-to-all; bench.py uses torch.distributed). */
/* counts[o] = records of the finished table run owned by rank o; the run's
 * packed bytes (kc_device_records) hold them as consecutive slices. */
kc_status kc_owner_counts(kc_ctx* ctx, uint32_t world, uint64_t* counts);
/* Replaces the finished ctx's table run by the sorted, summed merge of
 * n_records packed records (SortedKMerFile layout, any order, duplicates
 * allowed, u32 counts wrap) in device memory of the ctx's device. The ctx
 * stays finished; kc_reset starts a new count. KC_ERR_STATE before kc_finish
 * or when spill runs exist. */
kc_status kc_merge_records_device(kc_ctx* ctx, const void* d_packed, uint64_t n_records);
/* As kc_merge_records_device when the records are nruns runs laid out one
 * after another, each sorted by key (what an all-to-all of sorted runs
 * delivers): merged pairwise by merge path instead of re-sorted.
 * run_counts: host array of nruns record counts. */
kc_status kc_merge_runs_device(kc_ctx* ctx, const void* d_packed, const uint64_t* run_counts, uint32_t nruns);
/* The same exchange between n contexts of one process (the CLI's gpus=N
 * exchange=alltoall): context o ends up owning owner_of == o, so writing the
 * contexts' runs one after another in order is the whole SortedKMerFile.
 * Slices move by hipMemcpyPeer. Every ctx finished, same k, no spill runs. */
kc_status kc_exchange_contexts(kc_ctx* const* ctxs, uint32_t n);
/* Read-shard merge between n contexts of one process (the CLI's gpus=N,
 * exchange=none): every finished context's sorted run is copied to ctxs[0]'s
 * device (hipMemcpyPeer) and merged there by merge path (the device form of
 * the reference's KMerFileMergeHandler k-way merge,
 * KMerFileMergeHandler.cpp:49-100); ctxs[0] then holds the whole count.
 * KC_ERR_STATE when a context keeps spill runs in host memory (merge those
 * with kc_write_runs + kc_merge_files). */
kc_status kc_gather_contexts(kc_ctx* const* ctxs, uint32_t n);
/* Device->device copy on the ctx's stream (exchange staging). */
kc_status kc_copy_device(kc_ctx* ctx, void* d_dst, const void* d_src, uint64_t n_bytes);

/* ---- host merge of sorted runs (KMerFileMerger / KMerFileMergeHandler) ---- */
kc_status kc_merge_files(const char* const* inputs, uint32_t n_inputs, const char* output,
                         int64_t kmer_length, uint32_t merge_fan_in, uint32_t merge_threads);

/* The same merge shared by `parts` processes (the ranks of a read-shard job,
 * SURVEY §8e cfg3; the reference runs its merge groups concurrently,
 * KMerFileMergeHandler.cpp:41-123). Every process opens the same input files;
 * the key space is cut into `parts` ranges at keys chosen from the files by a
 * deterministic rule (no data exchange), and kc_merge_part_create merges range
 * `part` (by up to merge_threads threads) into host memory, reporting its
 * merged size. The caller gathers the sizes (an all-gather of one u64 per
 * process); part p is written at the sum of the sizes of parts 0..p-1 by
 * kc_merge_part_write, which also cuts the file to file_bytes (the sum of all
 * sizes; 0 = no cut). The parts written side by side are the bytes
 * kc_merge_files writes. kc_merge_part_destroy frees a part. */
typedef struct kc_merge_part kc_merge_part;
kc_status kc_merge_part_create(const char* const* inputs, uint32_t n_inputs, int64_t kmer_length, uint32_t part,
                               uint32_t parts, uint32_t merge_threads, kc_merge_part** out, uint64_t* n_bytes);
kc_status kc_merge_part_write(kc_merge_part* p, const char* output, uint64_t offset, uint64_t file_bytes);
void kc_merge_part_destroy(kc_merge_part* p);

/* ---- synthetic input (bench/test data; not on the counting path) ---------- */
uint64_t kc_synth_fastq_bytes(const kc_synth_spec* spec);
/* Writes the FASTQ text of spec into host memory (dst_bytes >= kc_synth_fastq_bytes). */
kc_status kc_synth_fastq_host(const kc_synth_spec* spec, char* dst, uint64_t dst_bytes);
/* Generates the same bytes directly in device memory of the ctx's device;
 * the buffer is owned by the ctx (freed by kc_synth_free or kc_destroy). */
kc_status kc_synth_fastq_device(kc_ctx* ctx, const kc_synth_spec* spec, void** d_out, uint64_t* n_bytes);
kc_status kc_synth_free(kc_ctx* ctx, void* d_buf);
/* Device->host copy helper for tests (no torch dependency). */
kc_status kc_copy_to_host(kc_ctx* ctx, void* dst, const void* d_src, uint64_t n_bytes);

#ifdef __cplusplus
}
#endif

#endif /* KC_H */
