// Host copy pool stress (kc_stage.cpp): par_memcpy of mixed sizes back to back
// through one Pool, checked byte for byte (tests/test_host.py builds and runs
// it; built with -fsanitize=thread it is a race check of the pool's handoff).
#include "kc_stage.h"
#include <cstdio>
#include <cstring>
#include <vector>
#include <cstdlib>
int main() {
    kc::Pool pool(16);
    std::vector<char> src((size_t)80 << 20), dst((size_t)80 << 20);
    for (size_t i = 0; i < src.size(); i++) src[i] = (char)(i * 131 + 7);
    size_t sizes[] = {100, 4096, 300000, 1u << 20, 7816500, (size_t)64 << 20, ((size_t)64 << 20) + 12345, 33554432};
    for (int rep = 0; rep < 2000; rep++) {
        size_t n = sizes[rep % 8];
        size_t off = (rep * 977) % 4096;
        if (off + n > src.size()) n = src.size() - off;
        memset(dst.data(), 0, n + off);
        kc::par_memcpy(&pool, dst.data() + off, src.data() + off, n);
        if (memcmp(dst.data() + off, src.data() + off, n) != 0) { printf("mismatch rep %d n %zu\n", rep, n); return 1; }
    }
    printf("ok\n");
    return 0;
}
