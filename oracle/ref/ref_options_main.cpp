// Driver (our code) for the reference's own, unmodified Options class
// (Options.cpp). Applies the argv prefix rules of getOptions (main.cpp:25-70)
// is NOT possible without main.cpp (it pulls KMerCounter.h -> TBB), so this
// only reports the Options constructor defaults for the CLI parity test.
// TEST INFRASTRUCTURE ONLY (oracle/_ref).
#include <cstdio>
#include <cinttypes>
#include "Options.h"

int main() {
    Options o;
    std::printf("kmerLength=%" PRId64 "\n", o.GetKmerLength());
    std::printf("gpuMemoryLimit=%" PRId64 "\n", o.GetGpuMemoryLimit());
    std::printf("noOfMergersAtOnce=%u\n", o.getNoOfMergersAtOnce());
    std::printf("noOfMergeThreads=%u\n", o.getNoOfMergeThreads());
    return 0;
}
