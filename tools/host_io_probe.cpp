// host_io_probe.cpp — measures the host side of the end-to-end path on the GPU
// box: PCIe copy rates (pinned / pageable, each direction, both at once), the
// host memcpy rate into pinned memory per thread count, a pipelined
// memcpy->pinned ring->DMA upload, and page-cache file write/read rates.
// Build: hipcc -O2 -std=c++17 tools/host_io_probe.cpp -o tools/host_io_probe -pthread
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/statfs.h>
#include <unistd.h>

#include <chrono>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__);     \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_memcpy(char* dst, const char* src, size_t n, int T) {
    if (T <= 1) {
        memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    size_t per = (n + T - 1) / T;
    for (int t = 0; t < T; t++) {
        size_t a = t * per, b = std::min(n, a + per);
        if (a >= b) break;
        th.emplace_back([=]() { memcpy(dst + a, src + a, b - a); });
    }
    for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
    const size_t G = 1ull << 30;
    const size_t N = (argc > 1 ? atoll(argv[1]) : 4) * G;
    cpu_set_t cs;
    sched_getaffinity(0, sizeof(cs), &cs);
    printf("cpus: sysconf=%ld affinity=%d\n", sysconf(_SC_NPROCESSORS_ONLN), CPU_COUNT(&cs));
    struct statfs sf;
    if (statfs("/tmp", &sf) == 0) printf("/tmp f_type=0x%lx (tmpfs=0x1021994, ext4=0xef53, xfs=0x58465342, overlay=0x794c7630)\n", (long)sf.f_type);
    if (statfs("/dev/shm", &sf) == 0) printf("/dev/shm f_type=0x%lx free=%.1f GB\n", (long)sf.f_type, sf.f_bavail * (double)sf.f_bsize / 1e9);
    CK(hipSetDevice(0));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    char *d, *d2, *hp, *hp2;
    CK(hipMalloc(&d, N));
    CK(hipMalloc(&d2, N));
    CK(hipHostMalloc(&hp, N, 0));
    CK(hipHostMalloc(&hp2, N, 0));
    char* pg = (char*)malloc(N);
    char* pg2 = (char*)malloc(N);
    memset(pg, 'A', N);
    memset(pg2, 'C', N);
    memset(hp, 'G', N);
    memset(hp2, 'T', N);
    auto rate = [&](const char* what, auto fn) {
        fn();  // warm
        CK(hipDeviceSynchronize());
        double t = now();
        fn();
        CK(hipDeviceSynchronize());
        double dt = now() - t;
        printf("%-44s %7.2f GB/s  (%.1f ms)\n", what, N / dt / 1e9, dt * 1e3);
        fflush(stdout);
    };
    rate("H2D pinned, one copy", [&]() { CK(hipMemcpyAsync(d, hp, N, hipMemcpyHostToDevice, s)); });
    rate("H2D pinned, 64 MiB copies", [&]() {
        for (size_t o = 0; o < N; o += 64 << 20) CK(hipMemcpyAsync(d + o, hp + o, 64 << 20, hipMemcpyHostToDevice, s));
    });
    rate("H2D pinned, 8 MiB copies", [&]() {
        for (size_t o = 0; o < N; o += 8 << 20) CK(hipMemcpyAsync(d + o, hp + o, 8 << 20, hipMemcpyHostToDevice, s));
    });
    rate("D2H pinned, one copy", [&]() { CK(hipMemcpyAsync(hp, d, N, hipMemcpyDeviceToHost, s)); });
    rate("H2D pageable, one copy", [&]() { CK(hipMemcpyAsync(d, pg, N, hipMemcpyHostToDevice, s)); });
    rate("D2H pageable, one copy", [&]() { CK(hipMemcpyAsync(pg, d, N, hipMemcpyDeviceToHost, s)); });
    rate("H2D + D2H pinned at once (per direction)", [&]() {
        CK(hipMemcpyAsync(d, hp, N, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(hp2, d2, N, hipMemcpyDeviceToHost, s2));
    });
    for (int T : {1, 2, 4, 8, 16, 24}) {
        char name[64];
        snprintf(name, sizeof(name), "memcpy pageable->pinned, %d threads", T);
        rate(name, [&]() { par_memcpy(hp, pg, N, T); });
    }
    for (int T : {4, 8, 16}) {
        // pipelined: T-thread memcpy into a ring of 4 x 64 MiB pinned slots, DMA each slot
        const size_t S = 64 << 20;
        hipEvent_t ev[4];
        for (auto& evb : ev) CK(hipEventCreateWithFlags(&evb, hipEventDisableTiming));
        char name[64];
        snprintf(name, sizeof(name), "pageable->ring(4x64MiB)->H2D, %d threads", T);
        rate(name, [&]() {
            int i = 0;
            for (size_t o = 0; o < N; o += S, i++) {
                int b = i & 3;
                CK(hipEventSynchronize(ev[b]));
                par_memcpy(hp + b * S, pg + o, S, T);
                CK(hipMemcpyAsync(d + o, hp + b * S, S, hipMemcpyHostToDevice, s));
                CK(hipEventRecord(ev[b], s));
            }
        });
    }
    for (int T : {1, 4, 8, 16}) {
        char path[64];
        snprintf(path, sizeof(path), "/tmp/kc_probe_%d.bin", (int)getpid());
        int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
        double t = now();
        std::vector<std::thread> th;
        size_t per = N / T;
        for (int k = 0; k < T; k++)
            th.emplace_back([=]() {
                for (size_t o = k * per; o < (k + 1) * per; o += 8 << 20) {
                    size_t m = std::min((size_t)8 << 20, (k + 1) * per - o);
                    if (pwrite(fd, hp + o, m, o) != (ssize_t)m) abort();
                }
            });
        for (auto& x : th) x.join();
        close(fd);
        double dt = now() - t;
        printf("%-44s %7.2f GB/s  (%.1f ms) [T=%d]\n", "file write (pwrite 8 MiB, page cache)", N / dt / 1e9, dt * 1e3, T);
        fd = open(path, O_RDONLY);
        t = now();
        th.clear();
        for (int k = 0; k < T; k++)
            th.emplace_back([=]() {
                for (size_t o = k * per; o < (k + 1) * per; o += 8 << 20) {
                    size_t m = std::min((size_t)8 << 20, (k + 1) * per - o);
                    if (pread(fd, hp2 + o, m, o) != (ssize_t)m) abort();
                }
            });
        for (auto& x : th) x.join();
        close(fd);
        dt = now() - t;
        printf("%-44s %7.2f GB/s  (%.1f ms) [T=%d]\n", "file read (pread 8 MiB, page cache)", N / dt / 1e9, dt * 1e3, T);
        unlink(path);
        fflush(stdout);
    }
    return 0;
}
