// Driver (our code) around the reference's own, unmodified merge classes
// (KMerFileMergeHandler.cpp, KMerFileMerger.cpp, SortedKMerFile.cpp compiled
// from /root/reference). Merges sorted run files into <outFile> the way the
// disabled spill path would (KMerCounter.cpp:57-59,111,164-165).
// TEST INFRASTRUCTURE ONLY (oracle/_ref). Usage:
//   ref_merge <outFile> <kmerLength> <fanIn> <threads> <run>...
// The handler never finishes with fewer runs than its fan-in (its Run loop only
// re-checks completion after launching a merge, KMerFileMergeHandler.cpp:54-84),
// so that case calls the final KMerFileMerger step directly, as Run does last.
#include <cstdio>
#include <cstdlib>
#include <list>
#include <string>
#include "KMerFileMergeHandler.h"
#include "KMerFileMerger.h"

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s <out> <k> <fanIn> <threads> <run>...\n", argv[0]);
        return 2;
    }
    std::string out = argv[1];
    uint64_t k = std::strtoull(argv[2], nullptr, 10);
    uint32_t fan = (uint32_t)std::atoi(argv[3]);
    uint32_t thr = (uint32_t)std::atoi(argv[4]);
    std::list<std::string> runs;
    for (int i = 5; i < argc; i++) runs.push_back(argv[i]);
    if (runs.size() < fan) {
        KMerFileMerger m(runs, out, k);
        m.Merge();
        return 0;
    }
    KMerFileMergeHandler h(out, k, fan, thr);
    for (auto& r : runs) h.AddFile(r);
    h.InputComplete();
    h.Start();
    h.Join();
    return 0;
}
