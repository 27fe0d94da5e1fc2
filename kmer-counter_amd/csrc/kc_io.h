// kc_io.h — host-side sorted-run I/O and k-way merge (internal to libkc_hip).
//
// Output format (SortedKMerFile, SortedKMerFile.cpp:18-124): records of W
// little-endian uint64 key words + little-endian uint32 count, rs = 8W+4 bytes,
// ascending by the key words compared as unsigned integers, word 0 first
// (KMerFileMerger::CheckLessThan, KMerFileMerger.cpp:98-108).
#pragma once
#include <stdint.h>

#include <fstream>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace kc {

// Byte buffers whose growth does not zero-fill (merge input and output
// buffers are written before they are read).
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInitAlloc<U>;
    };
    DefaultInitAlloc() noexcept = default;
    template <class U>
    DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
using ByteBuf = std::vector<uint8_t, DefaultInitAlloc<uint8_t>>;

// A sorted run: either a file or a host memory range.
struct RunSource {
    std::string path;              // non-empty: read from this file
    const uint8_t* mem = nullptr;  // else: this memory range
    uint64_t bytes = 0;
};

// Streams records of one run, folding consecutive equal keys the way
// SortedKMerFile::ReadKmer does (SortedKMerFile.cpp:57-82).
class RunReader {
  public:
    RunReader(const RunSource& src, int W);
    ~RunReader();
    RunReader(const RunReader&) = delete;
    RunReader& operator=(const RunReader&) = delete;
    bool ok() const { return ok_; }
    // Current (folded) record or nullptr at the end.
    const uint8_t* head() const { return have_ ? cur_.data() : nullptr; }
    void pop();

  private:
    bool raw_next(uint8_t* dst);
    void fill();
    int W_, rs_;
    bool ok_ = true, have_ = false;
    FILE* f_ = nullptr;
    const uint8_t* mem_ = nullptr;
    uint64_t mem_bytes_ = 0, mem_pos_ = 0;
    std::vector<uint8_t> buf_;
    size_t buf_pos_ = 0, buf_len_ = 0;
    std::vector<uint8_t> cur_, look_;
    bool look_valid_ = false;
};

// Buffered record writer (truncates the file).
class RunWriter {
  public:
    RunWriter(const std::string& path, int rs);
    ~RunWriter();
    bool ok() const { return f_ != nullptr && !err_; }
    void put(const uint8_t* rec);
    bool close();
    int error_number() const { return errno_; }  // errno of the first failure (0: none)

  private:
    void failed();
    FILE* f_ = nullptr;
    int rs_;
    bool err_ = false;
    int errno_ = 0;
    std::vector<uint8_t> buf_;
    size_t len_ = 0;
};

// k-way merge of sorted runs into `out`; equal keys are summed as uint32
// (KMerFileMerger::Merge, KMerFileMerger.cpp:49-96). Empty runs are skipped
// (the reference dereferences NULL on them, KMerFileMerger.cpp:58).
// On failure *err_no (if given) holds the errno of the failing call.
bool merge_runs(const std::vector<RunSource>& runs, const std::string& out, int W, int* err_no = nullptr);

// The same merge by up to `threads` threads over disjoint key ranges (each
// run's slice of a range found by binary search), written in place at each
// range's offset; runs may be files or memory. Same bytes as merge_runs.
bool merge_runs_parallel(const std::vector<RunSource>& runs, const std::string& out, int W, uint32_t threads,
                         int* err_no = nullptr);

// One part of a merge shared by `parts` processes over the same run files
// (cfg3's ranks): part boundaries are keys picked from the runs by a
// deterministic rule (no exchange between the processes), each part merged by
// up to `threads` threads into memory. The parts in order concatenate to
// merge_runs' bytes; part p's offset in the output is the sum of the sizes of
// parts 0..p-1 (the caller gathers them).
struct MergedPart {
    std::vector<ByteBuf> ranges;               // merged bytes, range by range in key order
    uint64_t bytes = 0;                        // sum of the ranges' sizes
    uint64_t in_records = 0;                   // input records of the part (all runs)
    uint32_t threads = 1;                      // writers of write_part_at
};
bool merge_runs_part(const std::vector<RunSource>& runs, int W, uint32_t part, uint32_t parts, uint32_t threads,
                     MergedPart* out, int* err_no = nullptr);
// Writes a part at `offset` of `path` (created if missing, not truncated);
// file_bytes > 0 cuts the file to that size (the node's total) afterwards.
bool write_part_at(const MergedPart& p, const std::string& path, uint64_t offset, uint64_t file_bytes,
                   int* err_no = nullptr);

// Merge tree with the reference handler's knobs (KMerFileMergeHandler.cpp):
// while more than fan_in runs remain, groups of fan_in runs are merged into
// temporary files "<tmp_prefix>.m<i>" by up to `threads` threads; the rest is
// merged into `out` (by merge_runs_parallel when threads > 1). The bytes of
// `out` do not depend on fan_in/threads.
bool merge_tree(const std::vector<RunSource>& runs, const std::string& out, int W, uint32_t fan_in,
                uint32_t threads, const std::string& tmp_prefix, std::string* err);

int key_compare(const uint8_t* a, const uint8_t* b, int W);

// KMerCounter::GetChunkSize (KMerCounter.cpp:193-212): bytes of sequence per
// reference chunk for read length L, k and gpuMemoryLimit.
int64_t reference_chunk_size(int64_t L, int64_t k, int64_t limit);

// Length of line 2 of a file: the read length L the reference takes per file
// (FASTQFileReader.cpp:31-35). 0 when the file has no second line.
int64_t file_line2_length(const std::string& path);

// The reference's chunker (FASTQFileReader::readData, FASTQFileReader.cpp:
// 49-89) driven the way InputFileHandler::read and KMerCounter::Start drive it
// (InputFileHandler.cpp:82-95, KMerCounter.cpp:123-143): the sequence lines
// (the line before each '+' line) concatenated without separators while the
// chunk has room; a record is lost at a chunk edge when its header is >= 2L
// long, exactly as in the reference. Used for inputMode=exact and as the
// fallback for input the GPU FASTQ decoder rejects.
class ExactChunker {
  public:
    ExactChunker(const std::string& path, int64_t L);
    bool done() const { return done_; }
    // Fills `chunk` with the next chunk's bytes; returns its size.
    int64_t next(int64_t cap, std::vector<char>& chunk);

  private:
    std::ifstream in_;
    int64_t size_ = 0, L_;
    bool done_ = false;
};

}  // namespace kc
