// Driver (our code) around the reference's own, unmodified input classes
// (InputFileHandler.cpp, FASTQFileReader.cpp, FASTQData.cpp compiled from
// /root/reference). It reproduces the chunk loop of KMerCounter::Start
// (KMerCounter.cpp:108-143) and writes every chunk that the reference would
// dispatch to processKMers into a binary file:
//   per chunk: int64 size, int64 lineLength, then `size` bytes.
// TEST INFRASTRUCTURE ONLY (oracle/_ref). Usage:
//   ref_reader <inputDir> <chunkSize> <outFile>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include "InputFileHandler.h"

int main(int argc, char** argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s <inputDir> <chunkSize> <outFile>\n", argv[0]);
        return 2;
    }
    int64_t chunk = std::strtoll(argv[2], nullptr, 10);
    std::FILE* out = std::fopen(argv[3], "wb");
    if (!out) return 3;
    InputFileHandler* h = new InputFileHandler(argv[1]);
    FASTQData* d = h->read(chunk);
    while (d != NULL) {
        int64_t L = h->getLineLength();
        int64_t size = d->getSize();
        // the dispatch condition of KMerCounter.cpp:130
        if (size > 0 && size >= L) {
            std::fwrite(&size, 8, 1, out);
            std::fwrite(&L, 8, 1, out);
            std::fwrite(d->getData(), 1, (size_t)size, out);
        }
        delete d;
        d = h->read(chunk);
    }
    std::fclose(out);
    delete h;
    return 0;
}
