// kc_stage.cpp — host staging of a device context: worker pool, pinned ring
// (PCIe upload / download), FASTQ file reader. See kc_stage.h.
#include "kc_stage.h"

#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>

namespace kc {

bool trace_on() {
    static const bool on = getenv("KC_TRACE") != nullptr;
    return on;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void trace(const char* fmt, ...) {
    if (!trace_on()) return;
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    fprintf(stderr, "kc-trace %.6f %s\n", now_s(), buf);
}

// ---------------------------------------------------------------------------
// Pool
// ---------------------------------------------------------------------------

Pool::Pool(int n_threads) {
    for (int i = 1; i < n_threads; i++) th_.emplace_back([this]() { loop(); });
}

Pool::~Pool() {
    {
        std::lock_guard<std::mutex> g(m_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
}

void Pool::loop() {
    uint64_t seen = 0;
    for (;;) {
        const std::function<void(int)>* fn;
        // back-to-back jobs (a caller's consecutive chunk copies) find the
        // worker spinning (up to ~0.5 ms) before it sleeps on the condition
        for (int spin = 0; spin < 20000 && gen_.load(std::memory_order_acquire) == seen &&
                           !stop_.load(std::memory_order_relaxed);
             spin++)
            __builtin_ia32_pause();
        {
            std::unique_lock<std::mutex> g(m_);
            cv_.wait(g, [&]() { return stop_.load() || gen_.load() != seen; });
            if (stop_) return;
            seen = gen_.load();
            fn = fn_;
            busy_++;
        }
        for (;;) {
            int i;
            {
                // only pieces of the job this worker joined: a worker that
                // joined after its job ended (fn null) must not take pieces of
                // the next one, whose counters the caller has reset
                std::lock_guard<std::mutex> g(m_);
                if (!fn || gen_.load() != seen || next_ >= n_) break;
                i = next_++;
            }
            (*fn)(i);
        }
        {
            std::lock_guard<std::mutex> g(m_);
            busy_--;
        }
        done_cv_.notify_all();
    }
}

void Pool::run(int n, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    if (th_.empty() || n == 1) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    {
        std::lock_guard<std::mutex> g(m_);
        fn_ = &fn;
        n_ = n;
        next_ = 0;
        gen_++;
    }
    cv_.notify_all();
    for (;;) {
        int i;
        {
            std::lock_guard<std::mutex> g(m_);
            if (next_ >= n_) break;
            i = next_++;
        }
        fn(i);
    }
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [&]() { return busy_ == 0; });
    fn_ = nullptr;
}

void par_memcpy(Pool* pool, void* dst, const void* src, size_t n) {
    const size_t kPiece = (size_t)1 << 18;
    int parts = 1;
    if (pool && n > kPiece)
        parts = n <= ((size_t)8 << 20) ? (int)((n + kPiece - 1) / kPiece) : pool->size();
    if (parts <= 1) {
        memcpy(dst, src, n);
        return;
    }
    const size_t per = ((n + parts - 1) / parts + 63) & ~(size_t)63;
    pool->run(parts, [&](int i) {
        const size_t a = (size_t)i * per;
        if (a >= n) return;
        memcpy((char*)dst + a, (const char*)src + a, std::min(per, n - a));
    });
}

bool host_is_pinned(const void* p) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// ---------------------------------------------------------------------------
// PinnedRing
// ---------------------------------------------------------------------------

PinnedRing::~PinnedRing() {
    (void)drain();
    for (auto e : ev_) (void)hipEventDestroy(e);
    for (auto p : slot_) (void)hipHostFree(p);
}

hipError_t PinnedRing::init(size_t slot_bytes, int slots) {
    if (ready()) return hipSuccess;
    slot_bytes_ = slot_bytes;
    for (int i = 0; i < slots; i++) {
        char* p = nullptr;
        hipEvent_t e = nullptr;
        hipError_t r = hipHostMalloc((void**)&p, slot_bytes, 0);
        if (r != hipSuccess) return r;
        r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (r != hipSuccess) {
            (void)hipHostFree(p);
            return r;
        }
        slot_.push_back(p);
        ev_.push_back(e);
        busy_.push_back(false);
    }
    return hipSuccess;
}

hipError_t PinnedRing::take(int i) {
    if (!busy_[i]) return hipSuccess;
    busy_[i] = false;
    return hipEventSynchronize(ev_[i]);
}

hipError_t PinnedRing::drain() {
    for (size_t i = 0; i < slot_.size(); i++) {
        hipError_t r = take((int)i);
        if (r != hipSuccess) return r;
    }
    return hipSuccess;
}

hipError_t PinnedRing::upload(void* d_dst, const void* src, size_t n, hipStream_t s, Pool* pool) {
    if (n == 0) return hipSuccess;
    if (host_is_pinned(src)) {
        // the caller's pinned buffer is read by the DMA itself: it must be
        // done before the buffer is handed back
        hipError_t r = hipMemcpyAsync(d_dst, src, n, hipMemcpyHostToDevice, s);
        return r != hipSuccess ? r : hipStreamSynchronize(s);
    }
    const int K = (int)slot_.size();
    for (size_t off = 0; off < n; off += slot_bytes_) {
        const size_t m = std::min(slot_bytes_, n - off);
        const int i = next_;
        next_ = (next_ + 1) % K;
        hipError_t r = take(i);
        if (r != hipSuccess) return r;
        par_memcpy(pool, slot_[i], (const char*)src + off, m);
        if ((r = hipMemcpyAsync((char*)d_dst + off, slot_[i], m, hipMemcpyHostToDevice, s)) != hipSuccess) return r;
        if ((r = hipEventRecord(ev_[i], s)) != hipSuccess) return r;
        busy_[i] = true;
    }
    return hipSuccess;
}

hipError_t PinnedRing::download(const void* d_src, size_t n, hipStream_t s,
                                const std::function<bool(const char*, size_t, size_t)>& sink) {
    if (n == 0) return hipSuccess;
    const int K = (int)slot_.size();
    hipError_t r = drain();
    if (r != hipSuccess) return r;
    const size_t np = (n + slot_bytes_ - 1) / slot_bytes_;
    // piece j lives in slot j % K; up to K - 1 DMAs run ahead of the sink
    const size_t ahead = (size_t)std::max(1, K - 1);
    size_t issued = 0;
    for (size_t j = 0; j < np; j++) {
        while (issued < np && issued < j + ahead) {
            const int i = (int)(issued % K);
            const size_t off = issued * slot_bytes_;
            if ((r = hipMemcpyAsync(slot_[i], (const char*)d_src + off, std::min(slot_bytes_, n - off),
                                    hipMemcpyDeviceToHost, s)) != hipSuccess)
                return r;
            if ((r = hipEventRecord(ev_[i], s)) != hipSuccess) return r;
            busy_[i] = true;
            issued++;
        }
        const int i = (int)(j % K);
        const double t0 = trace_on() ? now_s() : 0;
        if ((r = take(i)) != hipSuccess) return r;
        const double t1 = trace_on() ? now_s() : 0;
        const size_t off = j * slot_bytes_;
        const bool ok = sink(slot_[i], std::min(slot_bytes_, n - off), off);
        if (trace_on()) trace("download piece %zu: wait %.3f ms sink %.3f ms", j, (t1 - t0) * 1e3, (now_s() - t1) * 1e3);
        if (!ok) {
            (void)drain();
            return hipErrorUnknown;
        }
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------
// FASTQ blocks
// ---------------------------------------------------------------------------

size_t fastq_cut(const char* p, size_t n) {
    // candidates: positions q with p[q] == '@' and p[q - 1] == '\n', from the end
    size_t q = n;
    while (q > 1) {
        const char* hit = (const char*)memrchr(p, '@', q);
        if (!hit) return 0;
        q = (size_t)(hit - p);
        if (q == 0) return 0;
        if (p[q - 1] != '\n') continue;
        // lines q (header), q + 1 (sequence) must end inside the buffer and
        // line q + 2 must start there with '+'
        const char* e1 = (const char*)memchr(p + q, '\n', n - q);
        if (!e1) continue;
        const size_t l2 = (size_t)(e1 - p) + 1;
        if (l2 >= n) continue;
        const char* e2 = (const char*)memchr(p + l2, '\n', n - l2);
        if (!e2) continue;
        const size_t l3 = (size_t)(e2 - p) + 1;
        if (l3 >= n) continue;
        if (p[l3] == '+') return q;
    }
    return 0;
}

static const size_t kCarryMax = (size_t)64 << 20;  // longest record carried between blocks

size_t FastqFileReader::carry_bytes() { return kCarryMax; }

FastqFileReader::FastqFileReader(size_t block_bytes, const std::vector<char*>& bufs, int read_threads)
    : pool_(read_threads), block_(block_bytes), buf_(bufs) {}

FastqFileReader::~FastqFileReader() {
    {
        std::lock_guard<std::mutex> g(m_);
        stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
    if (fd_ >= 0) close(fd_);
}

bool FastqFileReader::open(const std::string& path, std::string* err) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) {
        *err = "cannot open " + path;
        return false;
    }
    off_t sz = lseek(fd_, 0, SEEK_END);
    if (sz < 0) {
        *err = "cannot size " + path;
        return false;
    }
    size_ = (uint64_t)sz;
    posix_fadvise(fd_, 0, 0, POSIX_FADV_SEQUENTIAL);
    if (size_ == 0) {
        done_ = true;
        return true;
    }
    block_ = (size_t)std::min<uint64_t>(block_, size_);
    // a file of one block needs one buffer
    if (block_ >= size_) buf_.resize(1);
    for (char* b : buf_)
        if (!b) {
            *err = "no pinned read buffers";
            return false;
        }
    len_.assign(buf_.size(), 0);
    cut_.assign(buf_.size(), 0);
    free_.assign(buf_.size(), true);
    th_ = std::thread([this]() { produce(); });
    return true;
}

// Fills buffer b: the tail of buffer prev (the previous block, -1 for the
// first), then up to block_ bytes of the file.
bool FastqFileReader::fill(int b, int prev) {
    size_t carry = 0;
    if (prev >= 0) {
        carry = len_[prev] - cut_[prev];
        if (carry > kCarryMax) {
            err_ = "a FASTQ record longer than 64 MiB";
            return false;
        }
        memcpy(buf_[b], buf_[prev] + cut_[prev], carry);
    }
    const size_t want = (size_t)std::min<uint64_t>(block_, size_ - pos_);
    const size_t kPiece = (size_t)8 << 20;
    const int parts = (int)std::max<size_t>(1, (want + kPiece - 1) / kPiece);
    bool ok = true;
    char* dst = buf_[b] + carry;
    const uint64_t at = pos_;
    pool_.run(parts, [&](int i) {
        const size_t a = (size_t)i * kPiece;
        const size_t m = std::min(kPiece, want - a);
        size_t got = 0;
        while (got < m) {
            ssize_t r = pread(fd_, dst + a + got, m - got, (off_t)(at + a + got));
            if (r <= 0) {
                ok = false;
                return;
            }
            got += (size_t)r;
        }
    });
    if (!ok) {
        err_ = "read error";
        return false;
    }
    if (trace_on()) trace("reader block %zu bytes at %llu", want, (unsigned long long)at);
    pos_ += want;
    len_[b] = carry + want;
    if (pos_ >= size_) {
        cut_[b] = len_[b];
    } else {
        cut_[b] = fastq_cut(buf_[b], len_[b]);
        // no second record start in the block: taken whole (the GPU index
        // rejects it if it is not whole records)
        if (cut_[b] == 0) cut_[b] = len_[b];
    }
    return true;
}

void FastqFileReader::produce() {
    int prev = -1;
    while (pos_ < size_) {
        int b = -1;
        {
            std::unique_lock<std::mutex> g(m_);
            // a buffer is refilled only after the next one took its tail: with
            // one buffer (a one-block file) there is no next
            cv_.wait(g, [&]() {
                if (stop_) return true;
                for (size_t i = 0; i < buf_.size(); i++)
                    if (free_[i] && (int)i != prev) return true;
                return false;
            });
            if (stop_) return;
            for (size_t i = 0; i < buf_.size(); i++)
                if (free_[i] && (int)i != prev) {
                    b = (int)i;
                    break;
                }
            free_[b] = false;
        }
        const bool ok = fill(b, prev);
        {
            std::lock_guard<std::mutex> g(m_);
            if (!ok) {
                done_ = true;
                free_[b] = true;
                break;
            }
            Block blk;
            blk.id = b;
            blk.p = buf_[b];
            blk.n = cut_[b];
            blk.index = produced_++;
            ready_.push_back(blk);
            // the previous buffer's tail is copied: it is free once its consumer releases it
        }
        cv_.notify_all();
        prev = b;
    }
    {
        std::lock_guard<std::mutex> g(m_);
        done_ = true;
    }
    cv_.notify_all();
}

bool FastqFileReader::next(Block* b) {
    std::unique_lock<std::mutex> g(m_);
    if (trace_on() && !(ready_head_ < ready_.size() || done_)) trace("consumer waits for a block");
    cv_.wait(g, [&]() { return ready_head_ < ready_.size() || done_; });
    if (ready_head_ >= ready_.size()) return false;
    *b = ready_[ready_head_++];
    return true;
}

void FastqFileReader::release(const Block& b) {
    {
        std::lock_guard<std::mutex> g(m_);
        if (b.id >= 0) free_[b.id] = true;
    }
    cv_.notify_all();
}

std::string FastqFileReader::error() {
    std::lock_guard<std::mutex> g(m_);
    return err_;
}

}  // namespace kc
