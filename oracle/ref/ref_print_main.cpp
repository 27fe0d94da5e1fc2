// Driver (our code) for the reference's own, unmodified KMerPrinter
// (KMerPrinter.cpp) — the `kmer-counter print <in> <out> <k>` subcommand of
// main.cpp:78-82. TEST INFRASTRUCTURE ONLY (oracle/_ref). Usage:
//   ref_print <in> <out-ignored> <k>
#include <cstdlib>
#include "KMerPrinter.h"

int main(int argc, char** argv) {
    if (argc != 4) return 2;
    KMerPrinter p(argv[1], argv[2], std::atoll(argv[3]));
    p.print();
    return 0;
}
