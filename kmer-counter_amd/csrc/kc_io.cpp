// kc_io.cpp — sorted-run reader/writer and the host k-way merge.
// Replaces KMerFileMerger / KMerFileMergeHandler / SortedKMerFile
// (KMerFileMerger.cpp:19-135, KMerFileMergeHandler.cpp:23-123,
// SortedKMerFile.cpp:18-124) with a heap merge over buffered streams.
#include "kc_io.h"

#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <queue>
#include <thread>

namespace kc {

static const size_t kIoBuf = 8u << 20;

int key_compare(const uint8_t* a, const uint8_t* b, int W) {
    for (int j = 0; j < W; j++) {
        uint64_t x, y;
        memcpy(&x, a + 8 * j, 8);
        memcpy(&y, b + 8 * j, 8);
        if (x != y) return x < y ? -1 : 1;
    }
    return 0;
}

RunReader::RunReader(const RunSource& src, int W) : W_(W), rs_(8 * W + 4) {
    cur_.resize(rs_);
    look_.resize(rs_);
    if (!src.path.empty()) {
        f_ = fopen(src.path.c_str(), "rb");
        if (!f_) {
            ok_ = false;
            return;
        }
        buf_.resize(kIoBuf - kIoBuf % rs_);
    } else {
        mem_ = src.mem;
        mem_bytes_ = src.bytes - src.bytes % rs_;
    }
    // prime: cur_ = first folded record
    if (raw_next(look_.data())) {
        look_valid_ = true;
        pop();
    }
}

RunReader::~RunReader() {
    if (f_) fclose(f_);
}

void RunReader::fill() {
    size_t keep = buf_len_ - buf_pos_;
    if (keep) memmove(buf_.data(), buf_.data() + buf_pos_, keep);
    size_t got = fread(buf_.data() + keep, 1, buf_.size() - keep, f_);
    buf_len_ = keep + got;
    buf_pos_ = 0;
}

bool RunReader::raw_next(uint8_t* dst) {
    if (f_) {
        if (buf_len_ - buf_pos_ < (size_t)rs_) fill();
        if (buf_len_ - buf_pos_ < (size_t)rs_) return false;
        memcpy(dst, buf_.data() + buf_pos_, rs_);
        buf_pos_ += rs_;
        return true;
    }
    if (mem_pos_ + rs_ > mem_bytes_) return false;
    memcpy(dst, mem_ + mem_pos_, rs_);
    mem_pos_ += rs_;
    return true;
}

// Moves the look-ahead into cur_ and folds following records with the same key.
void RunReader::pop() {
    if (!look_valid_) {
        have_ = false;
        return;
    }
    cur_.swap(look_);
    look_valid_ = false;
    have_ = true;
    while (raw_next(look_.data())) {
        if (memcmp(look_.data(), cur_.data(), 8 * W_) == 0) {
            uint32_t a, b;
            memcpy(&a, cur_.data() + 8 * W_, 4);
            memcpy(&b, look_.data() + 8 * W_, 4);
            a += b;
            memcpy(cur_.data() + 8 * W_, &a, 4);
            continue;
        }
        look_valid_ = true;
        break;
    }
}

RunWriter::RunWriter(const std::string& path, int rs) : rs_(rs) {
    f_ = fopen(path.c_str(), "wb");
    if (!f_) errno_ = errno;
    buf_.resize(kIoBuf - kIoBuf % rs);
}

void RunWriter::failed() {
    if (!err_) errno_ = errno ? errno : EIO;
    err_ = true;
}

RunWriter::~RunWriter() { close(); }

void RunWriter::put(const uint8_t* rec) {
    if (len_ + rs_ > buf_.size()) {
        if (f_ && fwrite(buf_.data(), 1, len_, f_) != len_) failed();
        len_ = 0;
    }
    memcpy(buf_.data() + len_, rec, rs_);
    len_ += rs_;
}

bool RunWriter::close() {
    if (!f_) return false;
    if (len_ && fwrite(buf_.data(), 1, len_, f_) != len_) failed();
    len_ = 0;
    if (fclose(f_) != 0) failed();
    f_ = nullptr;
    return !err_;
}

bool merge_runs(const std::vector<RunSource>& runs, const std::string& out, int W, int* err_no) {
    const int rs = 8 * W + 4;
    std::vector<RunReader*> rd;
    bool ok = true;
    for (const auto& r : runs) {
        RunReader* x = new RunReader(r, W);
        if (!x->ok()) {
            if (ok && err_no) *err_no = errno ? errno : EIO;
            ok = false;
        }
        rd.push_back(x);
    }
    RunWriter w(out, rs);
    if (!w.ok()) {
        if (ok && err_no) *err_no = w.error_number();
        ok = false;
    }
    if (ok) {
        auto greater = [&](int a, int b) {
            int c = key_compare(rd[a]->head(), rd[b]->head(), W);
            return c != 0 ? c > 0 : a > b;
        };
        std::priority_queue<int, std::vector<int>, decltype(greater)> pq(greater);
        for (int i = 0; i < (int)rd.size(); i++)
            if (rd[i]->head()) pq.push(i);
        std::vector<uint8_t> acc(rs);
        bool have = false;
        while (!pq.empty()) {
            int i = pq.top();
            pq.pop();
            const uint8_t* h = rd[i]->head();
            if (have && memcmp(acc.data(), h, 8 * W) == 0) {
                uint32_t a, b;
                memcpy(&a, acc.data() + 8 * W, 4);
                memcpy(&b, h + 8 * W, 4);
                a += b;
                memcpy(acc.data() + 8 * W, &a, 4);
            } else {
                if (have) w.put(acc.data());
                memcpy(acc.data(), h, rs);
                have = true;
            }
            rd[i]->pop();
            if (rd[i]->head()) pq.push(i);
        }
        if (have) w.put(acc.data());
        ok = w.close();
        if (!ok && err_no) *err_no = w.error_number();
    }
    for (auto* x : rd) delete x;
    return ok;
}

// ---------------------------------------------------------------------------
// Key-range parallel k-way merge (the last level of the merge tree).
//
// The reference merges two (noOfMergersAtOnce) files at a time, one thread per
// merge (KMerFileMergeHandler.cpp:49-100), so its last merge is one thread
// reading every record. Here the key space is cut into ranges of about
// kRangeRecs input records: a range starts at a splitter key, and each run's
// part of it is found by binary search (pread of single records), so equal
// keys always fall into one range and folding never crosses a range edge.
// `threads` workers take the ranges in key order, read each run's slice with
// pread (or from memory), merge and fold it in memory, and write the result
// at its offset in the output once the ranges before it are merged (the
// offsets are the prefix sums of the merged sizes). Same bytes as merge_runs.
// ---------------------------------------------------------------------------

static const uint64_t kRangeRecs = 4u << 20;

// input records per range; KC_MERGE_RANGE_RECS (a test hook, honoured only
// with KC_TEST_HOOKS=1 like the library's others) makes ranges small
static uint64_t range_recs() {
    const char* on = getenv("KC_TEST_HOOKS");
    const char* e = on && strcmp(on, "1") == 0 ? getenv("KC_MERGE_RANGE_RECS") : nullptr;
    const uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
    return v ? v : kRangeRecs;
}

namespace {

struct RunAccess {
    int fd = -1;
    const uint8_t* mem = nullptr;
    uint64_t n = 0;  // records
    int rs = 12;
    ~RunAccess() {
        if (fd >= 0) ::close(fd);
    }
    bool open_src(const RunSource& s, int rs_) {
        rs = rs_;
        if (!s.path.empty()) {
            fd = ::open(s.path.c_str(), O_RDONLY);
            if (fd < 0) return false;
            struct stat st;
            if (fstat(fd, &st) != 0) return false;
            n = (uint64_t)st.st_size / (uint64_t)rs;
        } else {
            mem = s.mem;
            n = s.bytes / (uint64_t)rs;
        }
        return true;
    }
    bool read(uint64_t i, uint64_t cnt, uint8_t* dst) const {
        const size_t want = (size_t)(cnt * (uint64_t)rs);
        if (mem) {
            memcpy(dst, mem + i * (uint64_t)rs, want);
            return true;
        }
        size_t got = 0;
        while (got < want) {
            ssize_t r = pread(fd, dst + got, want - got, (off_t)(i * (uint64_t)rs + got));
            if (r <= 0) {
                if (r < 0 && errno == EINTR) continue;
                if (r == 0) errno = EIO;
                return false;
            }
            got += (size_t)r;
        }
        return true;
    }
    // first record index in [lo, hi) whose key is >= key (hi if none)
    bool lower_bound(const uint8_t* key, int W, uint64_t lo, uint64_t hi, uint64_t* res) const {
        uint8_t rec[8 * 4 + 4];
        while (lo < hi) {
            const uint64_t mid = lo + (hi - lo) / 2;
            if (!read(mid, 1, rec)) return false;
            if (key_compare(rec, key, W) < 0)
                lo = mid + 1;
            else
                hi = mid;
        }
        *res = lo;
        return true;
    }
};

static inline uint64_t ld64(const uint8_t* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

// a < b on W key words (word 0 first, unsigned)
template <int W>
static inline bool key_less(const uint8_t* a, const uint8_t* b) {
    for (int j = 0; j < W; j++) {
        const uint64_t x = ld64(a + 8 * j), y = ld64(b + 8 * j);
        if (x != y) return x < y;
    }
    return false;
}

// Merges the slices (each sorted) into dst, folding equal keys (u32 sums; the
// sum is commutative, so which run's copy of a key comes first does not
// matter). The few runs of a merge level are scanned linearly for the
// smallest head (an exhausted run is swapped out), cheaper than a heap at
// m <= ~16 and without the heap's per-compare indirection.
template <int W>
static uint64_t merge_slices_w(const std::vector<const uint8_t*>& beg, const std::vector<const uint8_t*>& end,
                               uint8_t* dst) {
    const int rs = 8 * W + 4;
    std::vector<const uint8_t*> cur, lim;
    for (size_t i = 0; i < beg.size(); i++)
        if (beg[i] < end[i]) cur.push_back(beg[i]), lim.push_back(end[i]);
    int m = (int)cur.size();
    uint8_t* o = dst;
    while (m > 0) {
        int bi = 0;
        for (int i = 1; i < m; i++)
            if (key_less<W>(cur[i], cur[bi])) bi = i;
        const uint8_t* h = cur[bi];
        if (o != dst && memcmp(o - rs, h, 8 * W) == 0) {
            uint32_t a, b;
            memcpy(&a, o - 4, 4);
            memcpy(&b, h + 8 * W, 4);
            a += b;
            memcpy(o - 4, &a, 4);
        } else {
            memcpy(o, h, rs);
            o += rs;
        }
        cur[bi] += rs;
        if (cur[bi] >= lim[bi]) {
            cur[bi] = cur[m - 1];
            lim[bi] = lim[m - 1];
            m--;
        }
    }
    return (uint64_t)(o - dst);
}

// One-word keys (every k <= 32, cfg2/cfg3), at most M runs: a merge by
// output key rather than by input record. Each step takes the smallest head
// key of the live runs and consumes that key from every run whose head holds
// it, summing the counts; all M lanes do the same work each step (selects, no
// data-dependent branches), so the compiler keeps the heads in registers and
// nothing mispredicts. A read-shard job's runs cover one genome, so most keys
// are in most runs and a step emits one output record for ~M input records
// (the per-record min scan did ~M unpredictable compares per input record).
// An exhausted lane reads its last record again (a valid address) and stays
// dead; a key repeated inside one run (not written by the library, but valid
// SortedKMerFile input) is folded into the previous output record.
template <int M>
static uint64_t merge_keys_w1(const std::vector<const uint8_t*>& beg, const std::vector<const uint8_t*>& end,
                              uint8_t* dst) {
    static const uint8_t dead_rec[12] = {0};
    const uint8_t* cur[M];
    const uint8_t* lim[M];
    const uint8_t* tail[M];
    uint64_t hk[M];
    uint32_t hc[M];
    uint32_t al[M];
    int j = 0;
    for (size_t i = 0; i < beg.size(); i++)
        if (beg[i] < end[i]) {
            cur[j] = beg[i], lim[j] = end[i], tail[j] = end[i] - 12, al[j] = 1;
            j++;
        }
    for (; j < M; j++) cur[j] = lim[j] = tail[j] = dead_rec, al[j] = 0;
    uint32_t any = 0;
    for (int i = 0; i < M; i++) {
        const uint8_t* src = al[i] ? cur[i] : tail[i];
        hk[i] = ld64(src);
        memcpy(&hc[i], src + 8, 4);
        any |= al[i];
    }
    uint8_t* o = dst;
    uint64_t lastk = 0;
    while (any) {
        uint64_t mn = ~0ull;
        for (int i = 0; i < M; i++) {
            const uint64_t kk = al[i] ? hk[i] : ~0ull;
            mn = kk < mn ? kk : mn;
        }
        uint32_t sum = 0;
        any = 0;
        for (int i = 0; i < M; i++) {
            const bool e = al[i] && hk[i] == mn;
            sum += e ? hc[i] : 0u;
            const uint8_t* nx = cur[i] + (e ? 12 : 0);
            const uint32_t a = nx < lim[i] ? al[i] : 0u;
            const uint8_t* src = a ? nx : tail[i];
            cur[i] = nx;
            hk[i] = ld64(src);
            memcpy(&hc[i], src + 8, 4);
            al[i] = a;
            any |= a;
        }
        const bool fold = o != dst && mn == lastk;
        uint8_t* t = fold ? o - 12 : o;
        uint32_t prev;
        memcpy(&prev, fold ? o - 4 : dead_rec, 4);
        sum += fold ? prev : 0u;
        memcpy(t, &mn, 8);
        memcpy(t + 8, &sum, 4);
        o = t + 12;
        lastk = mn;
    }
    return (uint64_t)(o - dst);
}

static uint64_t merge_slices_w1(const std::vector<const uint8_t*>& beg, const std::vector<const uint8_t*>& end,
                                uint8_t* dst) {
    size_t m = 0;
    for (size_t i = 0; i < beg.size(); i++) m += beg[i] < end[i];
    if (m <= 4) return merge_keys_w1<4>(beg, end, dst);
    if (m <= 8) return merge_keys_w1<8>(beg, end, dst);
    if (m <= 16) return merge_keys_w1<16>(beg, end, dst);
    return merge_slices_w<1>(beg, end, dst);
}

static uint64_t merge_slices(const std::vector<const uint8_t*>& beg, const std::vector<const uint8_t*>& end, int W,
                             uint8_t* dst) {
    switch (W) {
    case 1: return merge_slices_w1(beg, end, dst);
    case 2: return merge_slices_w<2>(beg, end, dst);
    case 3: return merge_slices_w<3>(beg, end, dst);
    default: return merge_slices_w<4>(beg, end, dst);
    }
}

// Cuts run slices [lo, hi) into ranges of about range_recs() input records
// (bounds[r][i] = run i's first record of range r; the last entry is hi). A
// range is split at the middle key of the run holding most of its records;
// when that key is also the range's first key in every run (a long repeat),
// the cut moves past the repeat (upper bound), so no worker is handed the
// whole remainder. A range of one repeated key stays whole.
static bool plan_ranges(const std::vector<RunAccess>& acc, int W, const std::vector<uint64_t>& lo0,
                        const std::vector<uint64_t>& hi0, std::vector<std::vector<uint64_t>>* bounds, int* err_no,
                        uint64_t rr = 0) {
    const int m = (int)acc.size();
    if (rr == 0) rr = range_recs();
    using Rg = std::pair<std::vector<uint64_t>, std::vector<uint64_t>>;
    std::vector<Rg> todo{{lo0, hi0}}, done;
    uint8_t key[8 * 4 + 4], rec[8 * 4 + 4];
    auto io_fail = [&]() {
        if (err_no) *err_no = errno ? errno : EIO;
        return false;
    };
    while (!todo.empty()) {
        Rg rg = todo.back();
        todo.pop_back();
        uint64_t n = 0, best = 0;
        int bi = 0;
        for (int i = 0; i < m; i++) {
            const uint64_t c = rg.second[i] - rg.first[i];
            n += c;
            if (c > best) best = c, bi = i;
        }
        bool split = false;
        if (n > 2 * rr && best > 1) {
            if (!acc[bi].read(rg.first[bi] + best / 2, 1, key)) return io_fail();
            std::vector<uint64_t> cut(m);
            for (int i = 0; i < m; i++)
                if (!acc[i].lower_bound(key, W, rg.first[i], rg.second[i], &cut[i])) return io_fail();
            uint64_t left = 0, right = 0;
            for (int i = 0; i < m; i++) left += cut[i] - rg.first[i], right += rg.second[i] - cut[i];
            if (left == 0) {
                // the middle key is the smallest key of the range: cut after
                // every copy of it instead (first record with a larger key)
                for (int i = 0; i < m; i++) {
                    uint64_t a = rg.first[i], b = rg.second[i];
                    while (a < b) {
                        const uint64_t mid = a + (b - a) / 2;
                        if (!acc[i].read(mid, 1, rec)) return io_fail();
                        if (key_compare(rec, key, W) <= 0)
                            a = mid + 1;
                        else
                            b = mid;
                    }
                    cut[i] = a;
                }
                left = right = 0;
                for (int i = 0; i < m; i++) left += cut[i] - rg.first[i], right += rg.second[i] - cut[i];
            }
            if (left > 0 && right > 0) {
                todo.push_back({cut, rg.second});  // right half later: ranges come out in key order
                todo.push_back({rg.first, cut});
                split = true;
            }
        }
        if (!split) done.push_back(rg);
    }
    bounds->clear();
    for (auto& d : done) bounds->push_back(d.first);
    bounds->push_back(hi0);
    return true;
}

// Workers merging one range at a time need an input and a result buffer of up
// to ~2 range_recs() records each; the pool is capped so that those buffers
// stay within kMergeMemBudget however many CPUs the host has.
static const uint64_t kMergeMemBudget = 4ull << 30;

static uint32_t merge_workers(uint32_t threads, size_t ranges, int rs) {
    const uint64_t per = 2 * (2 * range_recs() * (uint64_t)rs);
    const uint64_t cap = std::max<uint64_t>(1, kMergeMemBudget / std::max<uint64_t>(1, per));
    uint64_t t = std::max<uint32_t>(1, threads);
    t = std::min<uint64_t>(t, cap);
    t = std::min<uint64_t>(t, std::max<size_t>(1, ranges));
    return (uint32_t)t;
}

// Merges every range of `bounds` by `threads` workers, in key order of
// completion commitment: `sink(r, data, bytes, offset)` receives range r's
// merged bytes and their offset from the first range (prefix sum of the
// merged sizes; called once per range, in any order, from the workers).
template <class Sink>
static bool merge_ranges(const std::vector<RunAccess>& acc, int W, const std::vector<std::vector<uint64_t>>& bounds,
                         uint32_t threads, uint64_t* total_bytes, int* err_no, Sink sink) {
    const int rs = 8 * W + 4;
    const int m = (int)acc.size();
    const size_t nr = bounds.size() - 1;
    std::mutex mu;
    std::condition_variable cv;
    size_t committed = 0;  // ranges whose output offset is known
    uint64_t next_off = 0;
    std::atomic<size_t> cursor(0);
    std::atomic<int> bad(0);
    auto work = [&]() {
        ByteBuf in, res;
        for (;;) {
            const size_t r = cursor.fetch_add(1);
            if (r >= nr) break;
            uint64_t cnt = 0;
            for (int i = 0; i < m; i++) cnt += bounds[r + 1][i] - bounds[r][i];
            in.resize((size_t)(cnt * (uint64_t)rs) + 1);
            res.resize((size_t)(cnt * (uint64_t)rs) + 1);
            std::vector<const uint8_t*> b(m), e(m);
            uint64_t pos = 0;
            bool ok = !bad.load();
            for (int i = 0; i < m && ok; i++) {
                const uint64_t c = bounds[r + 1][i] - bounds[r][i];
                if (c && !acc[i].read(bounds[r][i], c, in.data() + pos * (uint64_t)rs)) {
                    bad = errno ? errno : EIO;
                    ok = false;
                }
                b[i] = in.data() + pos * (uint64_t)rs;
                e[i] = b[i] + c * (uint64_t)rs;
                pos += c;
            }
            const uint64_t nbytes = ok ? merge_slices(b, e, W, res.data()) : 0;
            uint64_t off;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return committed == r; });
                off = next_off;
                next_off += nbytes;
                committed = r + 1;
            }
            cv.notify_all();
            if (ok && !sink(r, res, nbytes, off)) bad = errno ? errno : EIO;
        }
    };
    std::vector<std::thread> pool;
    const uint32_t nt = merge_workers(threads, nr, rs);
    for (uint32_t t = 0; t < nt; t++) pool.emplace_back(work);
    for (auto& t : pool) t.join();
    *total_bytes = next_off;
    if (bad.load()) {
        if (err_no) *err_no = bad.load();
        return false;
    }
    return true;
}

static bool pwrite_all(int fd, const uint8_t* p, uint64_t n, uint64_t off) {
    uint64_t put = 0;
    while (put < n) {
        ssize_t w = pwrite(fd, p + put, (size_t)(n - put), (off_t)(off + put));
        if (w <= 0) {
            if (w < 0 && errno == EINTR) continue;
            if (w == 0) errno = EIO;
            return false;
        }
        put += (uint64_t)w;
    }
    return true;
}

static bool open_runs(const std::vector<RunSource>& runs, int rs, std::vector<RunAccess>* acc, int* err_no) {
    *acc = std::vector<RunAccess>(runs.size());
    for (size_t i = 0; i < runs.size(); i++)
        if (!(*acc)[i].open_src(runs[i], rs)) {
            if (err_no) *err_no = errno ? errno : EIO;
            return false;
        }
    return true;
}

}  // namespace

bool merge_runs_parallel(const std::vector<RunSource>& runs, const std::string& out, int W, uint32_t threads,
                         int* err_no) {
    const int rs = 8 * W + 4;
    std::vector<RunAccess> acc;
    if (!open_runs(runs, rs, &acc, err_no)) return false;
    const int m = (int)acc.size();
    std::vector<uint64_t> lo(m, 0), hi(m);
    for (int i = 0; i < m; i++) hi[i] = acc[i].n;
    std::vector<std::vector<uint64_t>> bounds;
    if (!plan_ranges(acc, W, lo, hi, &bounds, err_no)) return false;
    int fd = ::open(out.c_str(), O_WRONLY | O_CREAT, 0644);
    if (fd < 0) {
        if (err_no) *err_no = errno;
        return false;
    }
    uint64_t total = 0;
    bool ok = merge_ranges(acc, W, bounds, threads, &total, err_no,
                           [&](size_t, ByteBuf& res, uint64_t n, uint64_t off) {
                               return pwrite_all(fd, res.data(), n, off);
                           });
    // written in place, cut to size (no truncation of an old file first)
    if (ok && ftruncate(fd, (off_t)total) != 0) {
        if (err_no) *err_no = errno;
        ok = false;
    }
    if (::close(fd) != 0 && ok) {
        if (err_no) *err_no = errno;
        ok = false;
    }
    return ok;
}

// ---------------------------------------------------------------------------
// One part of a merge shared by several processes (the ranks of a read-shard
// job, cfg3). Part boundaries are keys chosen from the runs themselves by a
// deterministic rule, so every process computes the same cuts from the same
// files without exchanging anything: boundary j (of parts - 1) is the median
// of the runs' keys at fraction j / parts of each run. A key's copies in every
// run fall on one side of each boundary, so the parts' merges concatenate to
// the whole merge.
// ---------------------------------------------------------------------------

bool merge_runs_part(const std::vector<RunSource>& runs, int W, uint32_t part, uint32_t parts, uint32_t threads,
                     MergedPart* out, int* err_no) {
    const int rs = 8 * W + 4;
    out->ranges.clear();
    out->bytes = 0;
    if (parts < 1 || part >= parts) {
        if (err_no) *err_no = EINVAL;
        return false;
    }
    std::vector<RunAccess> acc;
    if (!open_runs(runs, rs, &acc, err_no)) return false;
    const int m = (int)acc.size();
    uint64_t total = 0;
    for (int i = 0; i < m; i++) total += acc[i].n;
    // run i's first record of part j: 0 for j = 0, n_i for j = parts, else
    // the lower bound of boundary key K_j, the median of the runs' keys at
    // fraction j / parts of each run. Each run's candidate is non-decreasing
    // in j, so their median is, and the parts are disjoint key ranges in
    // order; only boundaries part and part + 1 are needed (O(m log n) reads).
    auto cut_at = [&](uint32_t j, std::vector<uint64_t>* cut) -> bool {
        cut->assign(m, 0);
        if (j == 0) return true;
        if (j >= parts) {
            for (int i = 0; i < m; i++) (*cut)[i] = acc[i].n;
            return true;
        }
        std::vector<std::vector<uint8_t>> cand;
        uint8_t key[8 * 4 + 4];
        for (int c = 0; c < m; c++) {
            if (acc[c].n == 0) continue;
            const uint64_t at = std::min<uint64_t>(acc[c].n - 1, (uint64_t)((long double)acc[c].n * j / parts));
            if (!acc[c].read(at, 1, key)) return false;
            cand.emplace_back(key, key + rs);
        }
        if (cand.empty()) return true;  // every run empty
        std::sort(cand.begin(), cand.end(), [&](const std::vector<uint8_t>& x, const std::vector<uint8_t>& y) {
            return key_compare(x.data(), y.data(), W) < 0;
        });
        const uint8_t* kj = cand[(cand.size() - 1) / 2].data();
        for (int i = 0; i < m; i++)
            if (!acc[i].lower_bound(kj, W, 0, acc[i].n, &(*cut)[i])) return false;
        return true;
    };
    std::vector<uint64_t> lo, hi;
    if (!cut_at(part, &lo) || !cut_at(part + 1, &hi)) {
        if (err_no) *err_no = errno ? errno : EIO;
        return false;
    }
    // sub-ranges small enough that every worker gets several (a part is a
    // fraction of the merge: with kRangeRecs ranges the last few would leave
    // most workers idle)
    uint64_t part_recs = 0;
    for (int i = 0; i < m; i++) part_recs += hi[i] - lo[i];
    const uint64_t rr = std::max<uint64_t>(1u << 16, std::min<uint64_t>(range_recs(),
                                                                       part_recs / (8ull * std::max(1u, threads))));
    std::vector<std::vector<uint64_t>> bounds;
    if (!plan_ranges(acc, W, lo, hi, &bounds, err_no, rr)) return false;
    out->ranges.assign(bounds.size() - 1, ByteBuf());
    uint64_t merged = 0;
    // a range's merged bytes stay in the worker's buffer, which the part
    // keeps (no copy; its unused tail is never touched)
    bool ok = merge_ranges(acc, W, bounds, threads, &merged, err_no,
                           [&](size_t r, ByteBuf& res, uint64_t n, uint64_t) {
                               res.resize((size_t)n);
                               out->ranges[r].swap(res);
                               return true;
                           });
    out->bytes = merged;
    out->threads = threads;
    for (int i = 0; i < m; i++) out->in_records += hi[i] - lo[i];
    return ok;
}

bool write_part_at(const MergedPart& p, const std::string& path, uint64_t offset, uint64_t file_bytes, int* err_no) {
    int fd = ::open(path.c_str(), O_WRONLY | O_CREAT, 0644);
    if (fd < 0) {
        if (err_no) *err_no = errno;
        return false;
    }
    // the ranges go out by up to p.threads writers (one thread's buffered
    // writes into a file run at ~4 GB/s on the GPU box, several at the file's
    // page-cache insert rate, ~10-12 GB/s)
    const size_t nr = p.ranges.size();
    std::vector<uint64_t> at(nr + 1, offset);
    for (size_t r = 0; r < nr; r++) at[r + 1] = at[r] + p.ranges[r].size();
    std::atomic<size_t> cursor(0);
    std::atomic<int> bad(0);
    auto work = [&]() {
        for (;;) {
            const size_t r = cursor.fetch_add(1);
            if (r >= nr || bad.load()) break;
            if (!pwrite_all(fd, p.ranges[r].data(), p.ranges[r].size(), at[r])) bad = errno ? errno : EIO;
        }
    };
    const uint32_t nt = (uint32_t)std::max<size_t>(1, std::min<size_t>(std::max<uint32_t>(1, p.threads), nr));
    if (nt == 1) {
        work();
    } else {
        std::vector<std::thread> pool;
        for (uint32_t t = 0; t < nt; t++) pool.emplace_back(work);
        for (auto& t : pool) t.join();
    }
    bool ok = !bad.load();
    if (!ok) errno = bad.load();
    // every part cuts the file to the node's total: idempotent, and no part
    // writes past it, so the order of the parts' truncations does not matter
    if (ok && file_bytes && ftruncate(fd, (off_t)file_bytes) != 0) ok = false;
    if (!ok && err_no) *err_no = errno ? errno : EIO;
    if (::close(fd) != 0 && ok) {
        if (err_no) *err_no = errno;
        ok = false;
    }
    return ok;
}

bool merge_tree(const std::vector<RunSource>& runs_in, const std::string& out, int W, uint32_t fan_in,
                uint32_t threads, const std::string& tmp_prefix, std::string* err) {
    if (fan_in < 2) fan_in = 2;
    if (threads < 1) threads = 1;
    std::vector<RunSource> runs;
    for (const auto& r : runs_in)
        if (!(r.path.empty() && r.bytes == 0)) runs.push_back(r);
    std::vector<std::string> temps;
    int round = 0;
    bool ok = true;
    while (ok && runs.size() > fan_in) {
        size_t groups = runs.size() / fan_in;
        std::vector<RunSource> next;
        std::vector<std::string> outs(groups);
        std::atomic<size_t> cursor(0);
        std::atomic<bool> good(true);
        std::atomic<int> bad_errno(0);
        auto work = [&]() {
            for (;;) {
                size_t g = cursor.fetch_add(1);
                if (g >= groups) break;
                std::vector<RunSource> grp(runs.begin() + g * fan_in, runs.begin() + (g + 1) * fan_in);
                int e = 0;
                if (!merge_runs(grp, outs[g], W, &e)) {
                    good = false;
                    bad_errno = e;
                }
            }
        };
        for (size_t g = 0; g < groups; g++) outs[g] = tmp_prefix + ".m" + std::to_string(round) + "_" + std::to_string(g);
        std::vector<std::thread> pool;
        for (uint32_t t = 0; t < threads && t < groups; t++) pool.emplace_back(work);
        for (auto& t : pool) t.join();
        if (!good) {
            ok = false;
            if (err) *err = std::string("merge of sorted runs into ") + tmp_prefix + "* failed: " + strerror(bad_errno.load());
            break;
        }
        for (size_t g = 0; g < groups; g++) {
            RunSource s;
            s.path = outs[g];
            next.push_back(s);
            temps.push_back(outs[g]);
        }
        for (size_t i = groups * fan_in; i < runs.size(); i++) next.push_back(runs[i]);
        runs.swap(next);
        round++;
    }
    if (ok) {
        int e = 0;
        ok = threads > 1 ? merge_runs_parallel(runs, out, W, threads, &e) : merge_runs(runs, out, W, &e);
        if (!ok && err) *err = "cannot write output file " + out + ": " + strerror(e);
    }
    for (const auto& t : temps) unlink(t.c_str());
    return ok;
}

int64_t reference_chunk_size(int64_t L, int64_t k, int64_t limit) {
    const int64_t kb = (k + 3) / 4;                   // bytes of a k-mer's bases
    const int64_t rec = ((kb + 7) / 8 + 1) * 8;       // rounded to words, plus one word
    const int64_t per = rec * (L - k + 1);            // record bytes of one read
    if (per - 1 == 0) return 0;
    return L * ((limit - L) / (per - 1));
}

int64_t file_line2_length(const std::string& path) {
    std::ifstream s(path.c_str());
    std::string l1, l2;
    std::getline(s, l1);
    std::getline(s, l2);
    return (int64_t)l2.size();
}

ExactChunker::ExactChunker(const std::string& path, int64_t L) : L_(L) {
    std::ifstream sz(path.c_str(), std::ios::ate | std::ios::binary);
    size_ = sz.is_open() ? (int64_t)sz.tellg() : 0;
    in_.open(path.c_str());
}

int64_t ExactChunker::next(int64_t cap, std::vector<char>& chunk) {
    chunk.resize((size_t)(cap > 0 ? cap : 0) + 1);
    int64_t used = 0;
    std::string prev, cur;
    std::getline(in_, prev);
    std::getline(in_, cur);
    while (!cur.empty() && used + (int64_t)prev.size() < cap) {
        if (cur[0] == '+') {
            memcpy(chunk.data() + used, prev.data(), prev.size());
            used += (int64_t)prev.size();
            std::getline(in_, prev);
            std::getline(in_, cur);
        } else {
            prev.swap(cur);
            std::getline(in_, cur);
        }
    }
    int64_t at = (int64_t)in_.tellg();
    if (at + L_ > size_ || used == 0) done_ = true;
    return used;
}

}  // namespace kc
