// kc_cli.cpp — the `kmer-counter` command line, a drop-in for the reference's
// main.cpp / Options / KMerCounter::Start / KMerPrinter.
//
//   kmer-counter kmerLength=31 inputFileLocation=DIR outputFile=FILE [key=value...]
//   kmer-counter print <in> <out-ignored> <k>
//
// Keys and defaults follow getOptions (main.cpp:25-70) and Options()
// (Options.cpp:16-22): every argv (argv[0] included) is prefix-matched, unknown
// keys are ignored, the last occurrence wins. Additive keys (not in the
// reference): gpus=N, exchange=none|alltoall (key-space exchange between the
// GPUs' runs, output by concatenation; runs that spilled fall back to the
// k-way merge), inputMode=auto|fastq|exact, tableBytes=B, quiet=1,
// readLengths=fixed|variable, outputFormat=sorted|dump.
//
// Input (InputFileHandler.cpp:22-47): every directory entry whose name does
// not start with '.', in readdir order; L of a file = length of its line 2
// (FASTQFileReader.cpp:31-35).
//   inputMode=fastq : the file goes to the GPU as raw FASTQ blocks
//                     (kc_count_fastq); it must be 4-line records of L bases.
//   inputMode=exact : the host rebuilds the reference's chunks exactly
//                     (FASTQFileReader::readData with the chunk size of
//                     KMerCounter::GetChunkSize) and sends them with
//                     kc_count_chunk — bit-exact even on malformed input.
//   inputMode=auto  : fastq when every block of the file validates, else exact.
//   readLengths=variable : reads of any length up to the file's longest
//                     sequence line, each counted as a reference read of its
//                     own length (KC_FLAG_VARLEN; SURVEY §8f row 1 — an
//                     extension, the reference has no defined result there).
//                     Always the fastq mode; a malformed file is an error.
// Output: the SortedKMerFile (sorted, deduplicated records), see include/kc.h.
//   outputFormat=dump : the record layout of the reference's active path,
//                     KMerCounter::DumpResults (KMerCounter.cpp:91-106): key
//                     word 0 (8 B LE) + count (4 B LE) per distinct key, for
//                     k > 32 truncated to word 0 as the reference does (keys
//                     that differ only past base 32 stay separate records).
//                     Records are in key order (the reference's TBB hash order
//                     is not reproducible); for k <= 32 the bytes equal the
//                     sorted output.
#include <dirent.h>
#include <fcntl.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <fstream>
#include <initializer_list>
#include <string>
#include <thread>
#include <vector>

#include "kc.h"

namespace {

struct Options {
    // main.cpp:27-30 overrides of the Options() constructor defaults (Options.cpp:16-22)
    std::string input_dir = "/home/jayangad/data/1";
    int64_t gpu_memory_limit = 100000000;
    std::string temp_dir = "/tmp/1";
    std::string output_file = "/tmp/2/output.bin";
    int64_t kmer_length = 32;
    uint32_t mergers_at_once = 2;
    uint32_t merge_threads = 2;
    // additive
    int gpus = 1;
    std::string exchange = "none";
    std::string input_mode = "auto";
    uint64_t table_bytes = 0;
    bool quiet = false;
    bool varlen = false;
    bool dump = false;
};

bool starts(const char* s, const char* p) { return strncmp(s, p, strlen(p)) == 0; }

Options parse(int argc, char** argv) {
    Options o;
    std::string read_lengths = "fixed", output_format = "sorted";
    for (int i = 0; i < argc; i++) {
        const char* a = argv[i];
        if (starts(a, "kmerLength=")) {
            o.kmer_length = (int64_t)strtoull(a + 11, nullptr, 10);
            printf("Updating KmerLength=%" PRId64 "\n", o.kmer_length);
        }
        if (starts(a, "gpuMemoryLimit=")) {
            o.gpu_memory_limit = (int64_t)strtoull(a + 15, nullptr, 10);
            printf("Updating Gpu Memory Limit=%" PRId64 "\n", o.gpu_memory_limit);
        }
        if (starts(a, "inputFileLocation=")) {
            o.input_dir = a + 18;
            printf("Updating Input File Location='%s'\n", o.input_dir.c_str());
        }
        if (starts(a, "tempFileLocation=")) {
            o.temp_dir = a + 17;
            printf("Updating Temp File Location='%s'\n", o.temp_dir.c_str());
        }
        if (starts(a, "outputFile=")) {
            o.output_file = a + 11;
            printf("Updating Output File='%s'\n", o.output_file.c_str());
        }
        if (starts(a, "noOfMergersAtOnce=")) {
            o.mergers_at_once = (uint32_t)atoi(a + 18);
            printf("Updating No Of Mergers At Once='%u'\n", o.mergers_at_once);
        }
        if (starts(a, "noOfMergeThreads=")) {
            o.merge_threads = (uint32_t)atoi(a + 17);
            printf("Updating No Of Merge Threads='%u'\n", o.merge_threads);
        }
        if (starts(a, "gpus=")) o.gpus = atoi(a + 5);
        if (starts(a, "inputMode=")) o.input_mode = a + 10;
        if (starts(a, "exchange=")) o.exchange = a + 9;
        if (starts(a, "tableBytes=")) o.table_bytes = strtoull(a + 11, nullptr, 10);
        if (starts(a, "quiet=")) o.quiet = atoi(a + 6) != 0;
        if (starts(a, "readLengths=")) read_lengths = a + 12;
        if (starts(a, "outputFormat=")) output_format = a + 13;
    }
    if (o.gpus < 1) o.gpus = 1;
    // additive keys take only their listed values (a typo must not select a
    // different mode silently)
    auto one_of = [](const char* key, const std::string& v, std::initializer_list<const char*> ok) {
        for (const char* x : ok)
            if (v == x) return;
        std::string all;
        for (const char* x : ok) all += std::string(all.empty() ? "" : "|") + x;
        fprintf(stderr, "kmer-counter: %s=%s: expected %s\n", key, v.c_str(), all.c_str());
        exit(1);
    };
    one_of("exchange", o.exchange, {"none", "alltoall"});
    one_of("inputMode", o.input_mode, {"auto", "fastq", "exact"});
    one_of("readLengths", read_lengths, {"fixed", "variable"});
    one_of("outputFormat", output_format, {"sorted", "dump"});
    o.varlen = read_lengths == "variable";
    o.dump = output_format == "dump";
    if (o.varlen && o.input_mode == "exact") {
        // the reference's chunker has no variable-length form
        fprintf(stderr, "kmer-counter: readLengths=variable cannot be combined with inputMode=exact\n");
        exit(1);
    }
    return o;
}

// ---------------------------------------------------------------------------
// print subcommand (KMerPrinter.cpp:35-91): each key word as 32 bases, then
// " <count>". Output file argument is ignored, as in the reference.
// ---------------------------------------------------------------------------
int do_print(const char* in, int64_t k) {
    int W = (int)(k / 32 + (k % 32 > 0 ? 1 : 0));
    int rs = 8 * W + 4;
    FILE* f = fopen(in, "rb");
    if (!f) return 0;  // the reference prints nothing for a missing file
    std::vector<unsigned char> buf((size_t)rs * 10000);
    std::string line;
    for (;;) {
        size_t got = fread(buf.data(), 1, buf.size(), f);
        if (got == 0) break;
        // the reference zero-fills its buffer, so a trailing partial record
        // prints with zero bytes past the end of the file
        if (got % rs) memset(buf.data() + got, 0, rs - got % rs);
        for (size_t off = 0; off < got; off += rs) {
            line.clear();
            for (int j = 0; j < W; j++) {
                uint64_t v;
                memcpy(&v, buf.data() + off + 8 * j, 8);
                for (int b = 0; b < 32; b++) line.push_back("ACGT"[(v >> (62 - 2 * b)) & 3]);
            }
            uint32_t c;
            memcpy(&c, buf.data() + off + 8 * W, 4);
            printf("%s %u\n", line.c_str(), c);
        }
        if (got < buf.size()) break;
    }
    fclose(f);
    return 0;
}

// ---------------------------------------------------------------------------
// input files
// ---------------------------------------------------------------------------

struct InputFile {
    std::string path;
    int64_t L = 0;
};

std::vector<InputFile> list_inputs(const std::string& dir) {
    std::vector<InputFile> v;
    DIR* d = opendir(dir.c_str());
    if (!d) {
        printf("Couldn't open directory : %s\n", dir.c_str());
        return v;
    }
    while (dirent* e = readdir(d)) {
        if (e->d_name[0] == '.') continue;  // InputFileHandler.cpp:27 skips "." prefixes
        InputFile f;
        f.path = dir + "/" + e->d_name;
        std::ifstream s(f.path.c_str());
        std::string l1, l2;
        std::getline(s, l1);
        std::getline(s, l2);
        f.L = (int64_t)l2.size();
        v.push_back(f);
    }
    closedir(d);
    return v;
}

// Longest sequence line (line 2 of every 4-line record) of a FASTQ text.
int64_t max_seq_line(const char* p, size_t n) {
    int64_t best = 0;
    size_t pos = 0, line = 0;
    while (pos < n) {
        const char* nl = (const char*)memchr(p + pos, '\n', n - pos);
        const size_t end = nl ? (size_t)(nl - p) : n;
        if (line % 4 == 1 && (int64_t)(end - pos) > best) best = (int64_t)(end - pos);
        line++;
        pos = end + 1;
    }
    return best;
}

struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    bool map(const std::string& path) {
        fd = open(path.c_str(), O_RDONLY);
        if (fd < 0) return false;
        struct stat st;
        if (fstat(fd, &st) != 0) return false;
        n = (size_t)st.st_size;
        if (n == 0) return true;
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) return false;
        p = (const char*)m;
        madvise(m, n, MADV_SEQUENTIAL);
        return true;
    }
    ~Mapped() {
        if (p) munmap((void*)p, n);
        if (fd >= 0) close(fd);
    }
};

// outputFormat=dump for k > 32: rewrites the SortedKMerFile in place as word 0
// + count per record (DumpResults, KMerCounter.cpp:96-103).
bool to_dump_format(const std::string& path, int W) {
    if (W == 1) return true;  // the same bytes
    const size_t rs = 8 * (size_t)W + 4;
    FILE* in = fopen(path.c_str(), "rb");
    if (!in) return false;
    const std::string tmp = path + ".dump.tmp";
    FILE* out = fopen(tmp.c_str(), "wb");
    if (!out) {
        fclose(in);
        return false;
    }
    std::vector<unsigned char> ib(rs * 65536), ob(12 * 65536);
    bool ok = true;
    for (;;) {
        const size_t got = fread(ib.data(), 1, ib.size(), in);
        const size_t nrec = got / rs;
        for (size_t r = 0; r < nrec; r++) {
            memcpy(ob.data() + 12 * r, ib.data() + rs * r, 8);
            memcpy(ob.data() + 12 * r + 8, ib.data() + rs * r + 8 * W, 4);
        }
        if (nrec && fwrite(ob.data(), 1, 12 * nrec, out) != 12 * nrec) ok = false;
        if (got < ib.size()) break;
    }
    fclose(in);
    if (fclose(out) || !ok) return false;
    return rename(tmp.c_str(), path.c_str()) == 0;
}

void die(kc_ctx* c, kc_status s, const char* what) {
    fprintf(stderr, "kmer-counter: %s: %s%s%s\n", what, kc_strerror(s), c ? ": " : "", c ? kc_last_error(c) : "");
    exit(1);
}

struct GpuWork {
    int gpu;
    kc_ctx* ctx = nullptr;
    std::vector<std::string> runs;
    kc_status status = KC_OK;
    std::string err;
};

}  // namespace

int main(int argc, char** argv) {
    printf("### kmer-counter application ###\n");
    if (argc == 5 && strncmp(argv[1], "print", 5) == 0) return do_print(argv[2], atoll(argv[4]));
    Options o = parse(argc, argv);
    fflush(stdout);
    if (o.kmer_length < 1 || o.kmer_length > KC_MAX_K) {
        fprintf(stderr, "kmer-counter: kmerLength must be in [1, %d]\n", KC_MAX_K);
        return 1;
    }
    std::vector<InputFile> files = list_inputs(o.input_dir);

    // one context per GPU; blocks are dealt round-robin (read-shard, no
    // collective). With fewer devices than gpus=N, contexts share devices.
    int ndev = kc_device_count();
    if (ndev <= 0) {
        fprintf(stderr, "kmer-counter: no HIP device\n");
        return 1;
    }
    std::vector<GpuWork> gw(o.gpus);
    for (int g = 0; g < o.gpus; g++) {
        kc_config cfg;
        memset(&cfg, 0, sizeof(cfg));
        cfg.device = g % ndev;
        cfg.kmer_length = o.kmer_length;
        cfg.line_length = files.empty() ? o.kmer_length : files[0].L;
        cfg.gpu_memory_limit = (uint64_t)o.gpu_memory_limit;
        cfg.table_bytes = o.table_bytes;
        cfg.temp_dir = o.temp_dir.c_str();
        cfg.flags = (o.quiet ? KC_FLAG_QUIET : KC_FLAG_NONE) | (o.varlen ? KC_FLAG_VARLEN : KC_FLAG_NONE);
        gw[g].gpu = g;
        kc_status s = kc_create(&gw[g].ctx, &cfg);
        if (s) die(nullptr, s, "cannot create device context");
    }

    // every file through kc_count_file: 256 MiB blocks read ahead into pinned
    // memory, decoded on the GPU, dealt to the contexts (read-shard, no
    // collective); auto mode falls back to the reference's chunker for a
    // file the GPU decoder rejects (KMerCounter.cpp:123-143,
    // FASTQFileReader.cpp:49-89)
    std::vector<kc_ctx*> ctxs;
    for (auto& w : gw) ctxs.push_back(w.ctx);
    const uint32_t mode = o.input_mode == "exact" ? KC_INPUT_EXACT
                          : o.input_mode == "fastq" ? KC_INPUT_FASTQ
                                                    : KC_INPUT_AUTO;
    for (const InputFile& file : files) {
        InputFile f = file;
        if (!o.varlen && f.L < o.kmer_length) continue;
        if (o.varlen) {
            // every read fits a slot of the file's longest sequence line
            Mapped m;
            if (!m.map(f.path)) die(nullptr, KC_ERR_IO, f.path.c_str());
            if (m.n == 0) continue;
            f.L = max_seq_line(m.p, m.n);
            if (f.L < o.kmer_length) continue;
        }
        uint64_t nr = 0;
        kc_status s = kc_count_file(ctxs.data(), (uint32_t)ctxs.size(), f.path.c_str(), f.L, mode, &nr);
        if (s) die(ctxs[0], s, f.path.c_str());
    }

    // finish every GPU, then write (one GPU) or merge the per-GPU runs
    for (auto& w : gw) {
        uint64_t n = 0;
        kc_status s = kc_finish(w.ctx, &n);
        if (s) die(w.ctx, s, "finish");
    }
    bool spilled = false;
    for (auto& w : gw) {
        kc_stats st;
        kc_get_stats(w.ctx, &st);
        spilled |= st.spill_runs > 0;
    }
    if (o.gpus == 1) {
        kc_status s = kc_write_output(gw[0].ctx, o.output_file.c_str(), o.mergers_at_once, o.merge_threads);
        if (s) die(gw[0].ctx, s, "write output");
    } else if (o.exchange == "alltoall" && !spilled) {
        // key-space exchange: context g owns the g-th key range, so the output
        // is the contexts' runs written one after another (no host merge)
        std::vector<kc_ctx*> cs;
        for (auto& w : gw) cs.push_back(w.ctx);
        kc_status s = kc_exchange_contexts(cs.data(), (uint32_t)cs.size());
        if (s) die(cs[0], s, "exchange");
        FILE* out = fopen(o.output_file.c_str(), "wb");
        if (!out) die(nullptr, KC_ERR_IO, o.output_file.c_str());
        std::vector<char> buf;
        for (auto& w : gw) {
            uint64_t n = 0;
            kc_finish(w.ctx, &n);
            uint64_t rs = 8 * (uint64_t)((o.kmer_length + 31) / 32) + 4;
            buf.resize(n * rs + 1);
            if ((s = kc_copy_records(w.ctx, buf.data(), n * rs))) die(w.ctx, s, "copy records");
            if (n && fwrite(buf.data(), 1, n * rs, out) != n * rs) die(nullptr, KC_ERR_IO, o.output_file.c_str());
        }
        if (fclose(out)) die(nullptr, KC_ERR_IO, o.output_file.c_str());
    } else {
        // read-shard: the contexts' runs merged on the first context's GPU
        // (kc_gather_contexts); contexts with spill runs in host memory take
        // the host k-way merge (KMerFileMergeHandler semantics)
        std::vector<kc_ctx*> cs;
        for (auto& w : gw) cs.push_back(w.ctx);
        kc_status s = kc_gather_contexts(cs.data(), (uint32_t)cs.size());
        if (s == KC_OK) {
            if ((s = kc_write_output(gw[0].ctx, o.output_file.c_str(), o.mergers_at_once, o.merge_threads)))
                die(gw[0].ctx, s, "write output");
        } else if (s == KC_ERR_STATE) {
            std::vector<std::string> all;
            for (auto& w : gw) {
                std::string prefix = o.temp_dir + "/kc_gpu" + std::to_string(w.gpu) + "." + std::to_string(getpid());
                uint32_t nr = 0;
                if ((s = kc_write_runs(w.ctx, prefix.c_str(), &nr))) die(w.ctx, s, "write runs");
                for (uint32_t i = 0; i < nr; i++) all.push_back(prefix + "." + std::to_string(i));
            }
            std::vector<const char*> ptrs;
            for (auto& p : all) ptrs.push_back(p.c_str());
            s = kc_merge_files(ptrs.data(), (uint32_t)ptrs.size(), o.output_file.c_str(), o.kmer_length,
                               o.mergers_at_once, o.merge_threads);
            for (auto& p : all) unlink(p.c_str());
            if (s) die(nullptr, s, "merge");
        } else {
            die(cs[0], s, "gather");
        }
    }
    if (o.dump && !to_dump_format(o.output_file, (int)((o.kmer_length + 31) / 32)))
        die(nullptr, KC_ERR_IO, o.output_file.c_str());
    for (auto& w : gw) {
        if (!o.quiet) {
            kc_stats st;
            kc_get_stats(w.ctx, &st);
            fprintf(stderr,
                    "gpu %d: reads=%" PRIu64 " windows=%" PRIu64 " valid=%" PRIu64 " distinct=%" PRIu64
                    " spilled=%" PRIu64 " runs=%" PRIu64 " insert_ms=%.3f\n",
                    w.gpu, st.reads, st.windows, st.valid_kmers, st.output_records, st.spilled_kmers, st.spill_runs,
                    st.insert_ms);
        }
        kc_destroy(w.ctx);
    }
    return 0;
}
