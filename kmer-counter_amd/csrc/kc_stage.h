// kc_stage.h — host side of the end-to-end path (internal to libkc_hip):
// the PCIe ingest and egress of a device context.
//
// The reference moves every chunk synchronously through pageable memory
// (cudaMemcpyAsync + sync, GPUHandler.cu:407-410, 460) from 8 host threads.
// Here one context owns
//   - Pool        : a few persistent worker threads (parallel memcpy / pread),
//   - PinnedRing  : pinned host slots; pageable input is copied into a slot by
//                   the pool while the previous slot's DMA runs, so a caller's
//                   buffer is free as soon as its bytes are in a slot (the
//                   upload itself stays asynchronous on the ctx stream), and
//                   device->host output is pipelined through the same slots
//                   into a sink (file or host memory);
//   - FastqFileReader : reads a FASTQ file into pinned blocks with the pool
//                   (pread), cut at record boundaries found locally (no scan of
//                   the whole file), the tail carried into the next block —
//                   replaces FASTQFileReader::readData's getline loop
//                   (FASTQFileReader.cpp:49-89) for the GPU-decoded path.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include <condition_variable>
#include <functional>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace kc {

// Host-side phase tracing (KC_TRACE=1): one line per phase on stderr with
// its wall time; the tracing subsystem the reference lacks.
bool trace_on();
double now_s();
void trace(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

class Pool {
  public:
    explicit Pool(int n_threads);
    ~Pool();
    int size() const { return (int)th_.size() + 1; }
    // fn(i) for i in [0, n): the calling thread takes part; returns when all are done
    void run(int n, const std::function<void(int)>& fn);

  private:
    void loop();
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* fn_ = nullptr;
    int n_ = 0, next_ = 0, busy_ = 0;
    std::atomic<uint64_t> gen_{0};  // job generation (written under m_, spun on without it)
    std::atomic<bool> stop_{false};
};

// memcpy of n bytes split over the pool: 256 KiB pieces up to 8 MiB (late
// workers take fewer pieces), else one equal part per thread
void par_memcpy(Pool* pool, void* dst, const void* src, size_t n);

// true when p is pinned (hipHostMalloc'ed or registered) host memory
bool host_is_pinned(const void* p);

class PinnedRing {
  public:
    ~PinnedRing();
    hipError_t init(size_t slot_bytes, int slots);
    bool ready() const { return !slot_.empty(); }
    size_t slot_bytes() const { return slot_bytes_; }
    // Host -> device copy of n bytes on stream s. Pinned sources are copied
    // directly; pageable ones through the slots. Returns when `src` may be
    // reused (the DMA may still be in flight; stream order covers later work).
    hipError_t upload(void* d_dst, const void* src, size_t n, hipStream_t s, Pool* pool);
    // Device -> host: n bytes from d_src, delivered in slot-sized pieces to
    // sink(piece, bytes, offset) in order while the next piece's DMA runs.
    // A false return from the sink stops the copy (returned as hipErrorUnknown).
    hipError_t download(const void* d_src, size_t n, hipStream_t s,
                        const std::function<bool(const char*, size_t, size_t)>& sink);
    // waits for every DMA that reads or writes the slots
    hipError_t drain();

  private:
    hipError_t take(int i);
    size_t slot_bytes_ = 0;
    std::vector<char*> slot_;
    std::vector<hipEvent_t> ev_;
    std::vector<bool> busy_;
    int next_ = 0;
};

// Finds the end of the last whole FASTQ record of p[0, n) that is followed by
// the start of another record: the largest position q (0 < q < n) where a
// line starting with '@' begins whose next-but-one line starts with '+' (a
// quality line starting with '@' is followed by a header and a sequence line,
// so it never passes). 0 when no such position exists.
size_t fastq_cut(const char* p, size_t n);

// FASTQ file -> pinned blocks of whole records. A producer thread reads the
// file in order into `nbuf` pinned buffers (pread split over a pool); each
// block ends at a record boundary and its tail starts the next block.
// Consumers (one per device context) take blocks in file order with next()
// and hand each back with release().
class FastqFileReader {
  public:
    struct Block {
        int id = -1;
        const char* p = nullptr;
        size_t n = 0;
        uint64_t index = 0;  // block number in the file
    };
    // bufs: `nbuf` pinned buffers of block_bytes + carry_bytes() each, owned by
    // the caller (pinning costs ~50 ms per GB: a context keeps them)
    FastqFileReader(size_t block_bytes, const std::vector<char*>& bufs, int read_threads);
    ~FastqFileReader();
    static size_t carry_bytes();
    bool open(const std::string& path, std::string* err);
    // next block in file order; false at the end of the file or on a read error
    bool next(Block* b);
    void release(const Block& b);
    // read error (empty when the file was read to its end)
    std::string error();
    uint64_t file_size() const { return size_; }

  private:
    void produce();
    bool fill(int b, int prev);
    Pool pool_;
    size_t block_;
    int fd_ = -1;
    uint64_t size_ = 0, pos_ = 0;
    std::vector<char*> buf_;
    std::vector<size_t> len_, cut_;
    std::vector<bool> free_;
    std::vector<Block> ready_;  // FIFO of filled blocks
    size_t ready_head_ = 0;
    bool done_ = false, stop_ = false;
    uint64_t produced_ = 0;
    std::string err_;
    std::mutex m_;
    std::condition_variable cv_;
    std::thread th_;
};

}  // namespace kc
