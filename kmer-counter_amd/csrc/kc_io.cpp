// kc_io.cpp — sorted-run reader/writer and the host k-way merge.
// Replaces KMerFileMerger / KMerFileMergeHandler / SortedKMerFile
// (KMerFileMerger.cpp:19-135, KMerFileMergeHandler.cpp:23-123,
// SortedKMerFile.cpp:18-124) with a heap merge over buffered streams.
#include "kc_io.h"

#include <errno.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
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
        ok = merge_runs(runs, out, W, &e);
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
