// host_io_probe2.cpp — second host probe: cold (never copied before) pageable
// buffers for H2D/D2H, and output-file write strategies (pwrite vs a shared
// mmap written by T threads, overlay /tmp vs tmpfs /dev/shm, D2H straight into
// the file mapping).
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/host_io_probe2.cpp -o tools/host_io_probe2 -pthread
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t err_ = (x);                                                         \
        if (err_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(err_), __LINE__); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par(int T, size_t n, const std::function<void(size_t, size_t)>& fn) {
    std::vector<std::thread> th;
    size_t per = ((n + T - 1) / T + 4095) & ~(size_t)4095;
    for (int t = 0; t < T; t++) {
        size_t a = t * per, b = std::min(n, a + per);
        if (a >= b) break;
        th.emplace_back([=, &fn]() { fn(a, b); });
    }
    for (auto& x : th) x.join();
}

static void report(const char* what, size_t n, double dt) {
    printf("%-58s %7.2f GB/s  (%.1f ms)\n", what, n / dt / 1e9, dt * 1e3);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const size_t G = 1ull << 30;
    const size_t N = (argc > 1 ? atoll(argv[1]) : 4) * G;
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    char* d;
    CK(hipMalloc(&d, N));
    CK(hipMemset(d, 7, N));
    char* hp;
    CK(hipHostMalloc(&hp, N, 0));
    memset(hp, 'G', N);
    for (size_t piece : {N, (size_t)1 << 30, (size_t)64 << 20}) {
        char* pg = (char*)malloc(N);
        memset(pg, 'A', N);  // touched, never used by HIP before
        double t = now();
        for (size_t o = 0; o < N; o += piece) CK(hipMemcpyAsync(d + o, pg + o, std::min(piece, N - o), hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        std::string w = "cold pageable H2D, pieces of " + std::to_string(piece >> 20) + " MiB";
        report(w.c_str(), N, now() - t);
        t = now();
        for (size_t o = 0; o < N; o += piece) CK(hipMemcpyAsync(pg + o, d + o, std::min(piece, N - o), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        w = "warm pageable D2H, pieces of " + std::to_string(piece >> 20) + " MiB";
        report(w.c_str(), N, now() - t);
        free(pg);
        pg = (char*)malloc(N);
        t = now();
        for (size_t o = 0; o < N; o += piece) CK(hipMemcpyAsync(pg + o, d + o, std::min(piece, N - o), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        w = "cold (untouched) pageable D2H, pieces of " + std::to_string(piece >> 20) + " MiB";
        report(w.c_str(), N, now() - t);
        free(pg);
    }
    for (const char* dir : {"/tmp", "/dev/shm"}) {
        std::string path = std::string(dir) + "/kc_probe2_" + std::to_string(getpid());
        for (int T : {1, 8, 16}) {
            int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0644);
            double t = now();
            par(T, N, [&](size_t a, size_t b) {
                for (size_t o = a; o < b; o += 8 << 20) {
                    size_t m = std::min((size_t)8 << 20, b - o);
                    if (pwrite(fd, hp + o, m, o) != (ssize_t)m) abort();
                }
            });
            close(fd);
            std::string w = std::string(dir) + " pwrite, T=" + std::to_string(T);
            report(w.c_str(), N, now() - t);
            unlink(path.c_str());
            fd = open(path.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0644);
            t = now();
            if (ftruncate(fd, N) != 0) abort();
            char* m = (char*)mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            if (m == MAP_FAILED) abort();
            par(T, N, [&](size_t a, size_t b) { memcpy(m + a, hp + a, b - a); });
            munmap(m, N);
            close(fd);
            w = std::string(dir) + " ftruncate+mmap memcpy, T=" + std::to_string(T);
            report(w.c_str(), N, now() - t);
            unlink(path.c_str());
        }
        {
            int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0644);
            double t = now();
            if (fallocate(fd, 0, 0, N) != 0) printf("fallocate failed on %s\n", dir);
            char* m = (char*)mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            par(16, N, [&](size_t a, size_t b) { memcpy(m + a, hp + a, b - a); });
            munmap(m, N);
            close(fd);
            report((std::string(dir) + " fallocate+mmap memcpy, T=16").c_str(), N, now() - t);
            unlink(path.c_str());
        }
        {
            // D2H straight into the file mapping (pageable destination), 256 MiB pieces
            int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0644);
            double t = now();
            if (ftruncate(fd, N) != 0) abort();
            char* m = (char*)mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            for (size_t o = 0; o < N; o += 256 << 20) CK(hipMemcpyAsync(m + o, d + o, 256 << 20, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            munmap(m, N);
            close(fd);
            report((std::string(dir) + " D2H into file mmap (256 MiB pieces)").c_str(), N, now() - t);
            unlink(path.c_str());
        }
        {
            // D2H into pinned ring (4 x 128 MiB) + 16-thread memcpy into the file mapping
            int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0644);
            double t = now();
            if (ftruncate(fd, N) != 0) abort();
            char* m = (char*)mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            const size_t S = 128 << 20;
            hipEvent_t ev[4];
            for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            size_t nch = (N + S - 1) / S;
            for (size_t i = 0; i < nch + 3; i++) {
                if (i < nch) {
                    int b = i & 3;
                    CK(hipMemcpyAsync(hp + b * S, d + i * S, S, hipMemcpyDeviceToHost, s));
                    CK(hipEventRecord(ev[b], s));
                }
                if (i >= 3 || i + 1 >= nch) {
                }
                if (i >= 3) {
                    size_t j = i - 3;
                    if (j < nch) {
                        int b = j & 3;
                        CK(hipEventSynchronize(ev[b]));
                        par(16, S, [&](size_t a, size_t bb) { memcpy(m + j * S + a, hp + b * S + a, bb - a); });
                    }
                }
            }
            munmap(m, N);
            close(fd);
            report((std::string(dir) + " D2H pinned ring -> 16-thread mmap memcpy").c_str(), N, now() - t);
            unlink(path.c_str());
        }
    }
    return 0;
}
