// host_io_probe3.cpp — output-file write strategies on the GPU box's /tmp:
// separate files in parallel (is the one-file rate an inode lock?), chunk
// size, fallocate first, O_DIRECT from pinned memory.
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/host_io_probe3.cpp -o tools/host_io_probe3 -pthread
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const std::string& what, size_t n, double dt) {
    printf("%-58s %7.2f GB/s  (%.1f ms)\n", what.c_str(), n / dt / 1e9, dt * 1e3);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const size_t G = 1ull << 30;
    const size_t N = (argc > 1 ? atoll(argv[1]) : 4) * G;
    const char* dir = argc > 2 ? argv[2] : "/tmp";
    char* hp = nullptr;
    if (hipHostMalloc(&hp, N, 0) != hipSuccess) return 1;
    memset(hp, 'G', N);
    std::string base = std::string(dir) + "/kc_probe3_" + std::to_string(getpid());
    for (int T : {1, 4, 8, 16}) {
        double t = now();
        std::vector<std::thread> th;
        size_t per = N / T;
        for (int k = 0; k < T; k++)
            th.emplace_back([&, k]() {
                std::string p = base + "." + std::to_string(k);
                int fd = open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
                for (size_t o = 0; o < per; o += 8 << 20) {
                    size_t m = std::min((size_t)8 << 20, per - o);
                    if (write(fd, hp + k * per + o, m) != (ssize_t)m) abort();
                }
                close(fd);
            });
        for (auto& x : th) x.join();
        report("separate files in parallel, T=" + std::to_string(T), N, now() - t);
        for (int k = 0; k < T; k++) unlink((base + "." + std::to_string(k)).c_str());
    }
    for (size_t chunk : {(size_t)1 << 20, (size_t)64 << 20, (size_t)512 << 20}) {
        double t = now();
        int fd = open(base.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
        for (size_t o = 0; o < N; o += chunk)
            if (write(fd, hp + o, std::min(chunk, N - o)) != (ssize_t)std::min(chunk, N - o)) abort();
        close(fd);
        report("one file, write() of " + std::to_string(chunk >> 20) + " MiB", N, now() - t);
        unlink(base.c_str());
    }
    for (int T : {1, 8}) {
        double t = now();
        int fd = open(base.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
        int fr = fallocate(fd, 0, 0, N);
        std::vector<std::thread> th;
        size_t per = N / T;
        for (int k = 0; k < T; k++)
            th.emplace_back([&, k]() {
                for (size_t o = k * per; o < (k + 1) * per; o += 8 << 20)
                    if (pwrite(fd, hp + o, 8 << 20, o) != (ssize_t)(8 << 20)) abort();
            });
        for (auto& x : th) x.join();
        close(fd);
        report("fallocate(" + std::to_string(fr) + ") + pwrite 8 MiB, T=" + std::to_string(T), N, now() - t);
        unlink(base.c_str());
    }
    for (int T : {1, 4, 8}) {
        double t = now();
        int fd = open(base.c_str(), O_CREAT | O_TRUNC | O_WRONLY | O_DIRECT, 0644);
        if (fd < 0) {
            printf("O_DIRECT open failed\n");
            break;
        }
        std::vector<std::thread> th;
        size_t per = N / T;
        bool bad = false;
        for (int k = 0; k < T; k++)
            th.emplace_back([&, k]() {
                for (size_t o = k * per; o < (k + 1) * per; o += 64 << 20)
                    if (pwrite(fd, hp + o, 64 << 20, o) != (ssize_t)(64 << 20)) bad = true;
            });
        for (auto& x : th) x.join();
        close(fd);
        report(std::string("O_DIRECT pwrite 64 MiB") + (bad ? " (FAILED)" : "") + ", T=" + std::to_string(T), N,
               now() - t);
        unlink(base.c_str());
    }
    // rewrite of an existing cached file (pages already allocated): the allocation share of the cost
    {
        int fd = open(base.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
        for (size_t o = 0; o < N; o += 64 << 20) (void)!write(fd, hp + o, 64 << 20);
        close(fd);
        double t = now();
        fd = open(base.c_str(), O_WRONLY, 0644);
        for (size_t o = 0; o < N; o += 64 << 20) (void)!pwrite(fd, hp + o, 64 << 20, o);
        close(fd);
        report("overwrite in place (pages cached), 64 MiB", N, now() - t);
        unlink(base.c_str());
    }
    return 0;
}
