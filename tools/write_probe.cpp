// write_probe: ways to write one 3.4 GB output file from host memory (the
// SortedKMerFile of cfg2), each into a fresh file (deleted before the next):
// buffered pwrite from 1 / 16 threads, MAP_SHARED mapping filled by 16 threads
// (plain and with MADV_POPULATE_WRITE first), O_DIRECT from 16 threads.
// Usage: write_probe DIR [GB] [threads]
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/statfs.h>
#include <sys/utsname.h>
#include <unistd.h>

#include <atomic>
#include <functional>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void par(int T, const std::function<void(int)>& f) {
    std::vector<std::thread> th;
    for (int i = 1; i < T; i++) th.emplace_back(f, i);
    f(0);
    for (auto& t : th) t.join();
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    const double gb = argc > 2 ? atof(argv[2]) : 3.4;
    const int T = argc > 3 ? atoi(argv[3]) : 16;
    const size_t n = ((size_t)(gb * 1e9) + 4095) & ~(size_t)4095;
    const size_t piece = (size_t)8 << 20;
    struct statfs sf;
    statfs(dir.c_str(), &sf);
    struct utsname u;
    uname(&u);
    printf("{\"dir\": \"%s\", \"fs_type\": \"0x%lx\", \"kernel\": \"%s\", \"bytes\": %zu, \"threads\": %d}\n", dir.c_str(),
           (unsigned long)sf.f_type, u.release, n, T);
    char* src = (char*)aligned_alloc(4096, n);
    par(T, [&](int i) {
        size_t a = n / T * i, b = i == T - 1 ? n : n / T * (i + 1);
        for (size_t j = a; j < b; j++) src[j] = (char)(j * 131);
    });
    const std::string path = dir + "/kc_write_probe.bin";
    auto report = [&](const char* what, double t0, double t1, double t2, int err) {
        printf("{\"method\": \"%s\", \"GBps\": %.2f, \"write_ms\": %.1f, \"close_ms\": %.1f, \"errno\": %d}\n", what,
               n / (t2 - t0) / 1e9, (t1 - t0) * 1e3, (t2 - t1) * 1e3, err);
        fflush(stdout);
        unlink(path.c_str());
    };
    for (int rep = 0; rep < 2; rep++) {
        // (a) buffered pwrite, one thread
        {
            double t0 = now();
            int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
            int err = fallocate(fd, 0, 0, n) ? errno : 0;
            for (size_t off = 0; off < n; off += piece) pwrite(fd, src + off, std::min(piece, n - off), off);
            double t1 = now();
            close(fd);
            report("pwrite_1thread", t0, t1, now(), err);
        }
        // (b) buffered pwrite, T threads, disjoint pieces of one file
        {
            double t0 = now();
            int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
            int err = fallocate(fd, 0, 0, n) ? errno : 0;
            std::atomic<size_t> next(0);
            par(T, [&](int) {
                for (;;) {
                    size_t off = next.fetch_add(piece);
                    if (off >= n) break;
                    pwrite(fd, src + off, std::min(piece, n - off), off);
                }
            });
            double t1 = now();
            close(fd);
            report("pwrite_Tthreads", t0, t1, now(), err);
        }
        // (c, d) MAP_SHARED mapping filled by T threads (d: MADV_POPULATE_WRITE per piece first)
        for (int pop = 0; pop < 3; pop++) {
            double t0 = now();
            int fd = open(path.c_str(), O_CREAT | O_RDWR | O_TRUNC, 0644);
            int err = fallocate(fd, 0, 0, n) ? errno : 0;
            if (ftruncate(fd, n)) err = errno;
            char* m = (char*)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            if (m == MAP_FAILED) {
                printf("mmap failed %d\n", errno);
                close(fd);
                continue;
            }
            std::atomic<int> perr(0);
            std::atomic<size_t> next(0);
            par(T, [&](int) {
                for (;;) {
                    size_t off = next.fetch_add(piece);
                    if (off >= n) break;
                    size_t len = std::min(piece, n - off);
                    if (pop == 1 && madvise(m + off, len, 23 /* MADV_POPULATE_WRITE */)) perr = errno;
                    memcpy(m + off, src + off, len);
                }
            });
            double t1 = now();
            munmap(m, n);
            close(fd);
            const char* names[3] = {"mmap_Tthreads", "mmap_populate_write_Tthreads", "mmap_Tthreads_nofallocate"};
            report(names[pop], t0, t1, now(), pop == 1 ? perr.load() : err);
            if (pop == 1 && perr) printf("{\"note\": \"MADV_POPULATE_WRITE errno %d\"}\n", perr.load());
        }
        // (e) O_DIRECT, T threads
        {
            double t0 = now();
            int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC | O_DIRECT, 0644);
            int err = fd < 0 ? errno : 0;
            if (fd >= 0) {
                if (fallocate(fd, 0, 0, n)) err = errno;
                std::atomic<size_t> next(0);
                std::atomic<int> werr(0);
                par(T, [&](int) {
                    for (;;) {
                        size_t off = next.fetch_add(piece);
                        if (off >= n) break;
                        if (pwrite(fd, src + off, std::min(piece, n - off), off) < 0) werr = errno;
                    }
                });
                if (werr) err = werr;
                double t1 = now();
                close(fd);
                report("odirect_Tthreads", t0, t1, now(), err);
            } else {
                report("odirect_Tthreads(open failed)", t0, t0, now(), err);
            }
        }
    }
    free(src);
    return 0;
}
