/*
 * fk_main.cpp — ./findKmer, the drop-in host program.
 *
 * Mirrors the reference main() (findKmer/src/findKmer.cpp:1292-1379): the same
 * argv grammar (parse_arguments :394-490), defaults (:74-82, set_default_conf
 * :257-305), output file names, stdout/stderr text and exit codes, so that
 * k6thru11fullANDupstream.sh and users can call it unchanged.  The scan
 * (findKmer() :962-1069) runs on the GPU through the C-ABI in
 * include/findkmer.h; the CSV and stats files are written by fk_writer.cpp.
 *
 * Deliberate differences:
 *  - the reference always crashes in free() after writing its outputs
 *    (:1370, exit 134/139); this program exits 0 there;
 *  - a missing option value makes the reference re-print the usage forever
 *    (`while (!parse_arguments(...)) usage();`, :1302); this program prints it
 *    once more and exits 1;
 *  - an input ending inside a '>' line makes the reference spin forever
 *    (:1005); this program reports it and exits 1.
 * Extensions:
 *  - with -q 1 the file is first made device-resident by parallel pread into
 *    pinned buffers + async H2D (fk_input_load), then scanned in one feed;
 *    -q 0 (per-record progress lines) and non-regular files stream it in
 *    256 MiB pieces (FINDKMER_INGEST=stream forces that path);
 *  - --sweep KMAX: run k, k+1, ..., KMAX over one read of the file, writing
 *    each k's files exactly as separate invocations would (what
 *    k6thru11fullANDupstream.sh does with six processes per file).
 */
#include "findkmer.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <sys/mman.h>
#include <sys/stat.h>

#include <iostream>
#include <string>
#include <vector>

/* FINDKMER_TIMES=1: wall time of each phase of a run on stderr (off by
   default: stderr stays byte-identical to the reference's) */
static double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}
static bool g_times = false;
static void phase(int k, const char *what, double &t0) {
    if (!g_times) return;
    const double t = now_s();
    fprintf(stderr, "[findKmer k=%d] %-16s %9.3f ms\n", k, what, (t - t0) * 1e3);
    t0 = t;
}

#define DEFAULT_SEQUENCE_FILE_NAME "test.txt"
#define DEFAULT_K_VALUE 7
#define OUT_FILE_COLUMN_HEADERS "Sequence, Shannon Entropy h, Shannon Entropy H, Frequency, Z score"
#define DEFAULT_SUPPRESS_OUTPUT_VALUE 0
#define DEFAULT_Z_THRESHOLD_ENABLE 0
#define DEFAULT_Z_THRESHOLD 1000

static struct conf {
    const char *sequence_file;
    FILE *sequence_file_pointer;
    std::string out_file;
    bool out_set;
    FILE *out_file_pointer;
    int k;
    int suppressOutputEnable;
    long double zThreshold;
    int zThresholdEnable;
} config;

static int sweep_kmax = -1;          /* --sweep KMAX (extension) */
static fk_input *g_input = nullptr;  /* device-resident copy of the sequence file */
static bool g_input_tried = false;
static int g_device = -1;            /* fk_device_select's choice */

static void check_file(const char *filename, const char *mode) {   /* :233-242 */
    FILE *file = fopen(filename, mode);
    if (file == NULL) {
        fprintf(stderr, "Unable to open file %s in %s mode\nFile MUST be in current directory.\n",
                filename, mode);
        exit(EXIT_FAILURE);
    } else
        fclose(file);
}

static void init_conf() {                                           /* :246-255 */
    config.sequence_file = NULL;
    config.sequence_file_pointer = NULL;
    config.out_set = false;
    config.out_file_pointer = NULL;
    config.k = 0;
    config.suppressOutputEnable = -1;
    config.zThresholdEnable = -1;
    config.zThreshold = -1;
}

static void set_default_conf() {                                    /* :257-305 */
    if (!config.sequence_file) config.sequence_file = DEFAULT_SEQUENCE_FILE_NAME;
    if (!config.k) config.k = DEFAULT_K_VALUE;
    if (config.suppressOutputEnable < 0) config.suppressOutputEnable = DEFAULT_SUPPRESS_OUTPUT_VALUE;
    if (config.zThresholdEnable < 0) {
        config.zThresholdEnable = DEFAULT_Z_THRESHOLD_ENABLE;
        config.zThreshold = DEFAULT_Z_THRESHOLD;
    }
    if (!config.out_set) {
        char buf[64];
        snprintf(buf, sizeof buf, "%d", config.k);
        config.out_file = std::string(buf) + "mer_Historam_Of_" + config.sequence_file +
                          (config.zThresholdEnable == 0 ? "" : "zScoreFiltered") + ".csv";
        config.out_set = true;
    }
}

static void print_conf(int argc) {                                  /* :307-364 */
    fprintf(stdout, "\nATTEMPTING CONFIGURATION: \n");
    set_default_conf();
    if (config.sequence_file) fprintf(stdout, "- sequence_file file: %s\n", config.sequence_file);
    fprintf(stdout, "- export file: %s\n", config.out_file.c_str());
    if (config.k) fprintf(stdout, "- k size: %d\n", config.k);
    fprintf(stdout, "- %s\n",
            config.suppressOutputEnable > 0 ? "Suppressing file read output and breaks."
                                            : "Showing DNA Sequence identifier and allowing breaks.");
    fprintf(stdout, "- Z score filtering is %s", config.zThresholdEnable ? "enabled" : "disabled");
    if (config.zThresholdEnable > 0) fprintf(stdout, "\n    with threshold of %LG", config.zThreshold);
    fprintf(stdout, ".\n");
    if (config.suppressOutputEnable == 0 && argc < 2) {
        fprintf(stdout, "Press enter to proceed with this configuration.");
        getchar();
    }
    if (config.k < 0 || config.k > 20) {
        fprintf(stderr, "%d is not a valid value for k. Please select a number greater than zero\n", config.k);
        exit(EXIT_FAILURE);
    }
    if ((config.sequence_file_pointer = fopen(config.sequence_file, "r")) == NULL) {
        fprintf(stderr, "Sequence file failed to open\n\n");
        exit(EXIT_FAILURE);
    }
    if ((config.out_file_pointer = fopen(config.out_file.c_str(), "w")) != NULL) {
        fprintf(config.out_file_pointer, OUT_FILE_COLUMN_HEADERS);
    } else {
        fprintf(stderr, "Out file failed to open\nFile MUST be in current directory.\n");
        exit(EXIT_FAILURE);
    }
    fprintf(stdout, "Sequence file and out file opened properly\n");
    fprintf(stdout, "\n");
}

static void usage() {                                               /* :366-393 */
    fprintf(stdout, "\n");
    fprintf(stdout, "Usage: findKmer [options]\n");
    fprintf(stdout,
            "             [--parse|-p <sequence_file.txt>] \n"
            "               File with DNA sequence data.\n"
            "               File must be in current directory.\n"
            "               Parser follows .fas and .fa formats\n"
            "                Default is %s.\n\n",
            DEFAULT_SEQUENCE_FILE_NAME);
    fprintf(stdout,
            "             [--export|-e  <out_file.csv>] \n"
            "               File to output histogram data to.\n"
            "                Default output file name is dynamic.\n\n");
    fprintf(stdout,
            "             [--ksize|-k  <k>] \n"
            "               Size of sequence for histogram.\n"
            "                Default is %d.\n\n",
            DEFAULT_K_VALUE);
    fprintf(stdout,
            "             [--quiet|-q  < 0 for FALSE | 1 for TRUE >] \n"
            "               Suppress file read output and breaks.\n"
            "                Default is %s.\n\n",
            DEFAULT_SUPPRESS_OUTPUT_VALUE ? "true" : "false");
    long double tempzThreshold = DEFAULT_Z_THRESHOLD;
    fprintf(stdout,
            "             [--zthreshold|-z  < Threshold_for_Z >] \n"
            "               Suppress sequences with Z scores < threshold.\n"
            "                Default is %s with a value of %LG.\n\n",
            DEFAULT_Z_THRESHOLD_ENABLE ? "enabled" : "disabled", tempzThreshold);
    fprintf(stdout, "\n");
}

static int parse_arguments(int argc, char **argv) {                 /* :394-490 */
    int i = 1;
    if (argc < 2) return 1;
    while (i < argc) {
        if (strcmp(argv[i], "-h") == 0 || strcmp(argv[i], "--help") == 0) {
            exit(1);
        } else if (strcmp(argv[i], "-e") == 0 || strcmp(argv[i], "--export") == 0) {
            i++;
            if (i == argc) {
                fprintf(stderr, "Export file name missing.\n");
                return 0;
            }
            check_file(argv[i], "w");
            config.out_file = argv[i];
            config.out_set = true;
        } else if (strcmp(argv[i], "-p") == 0 || strcmp(argv[i], "--parse") == 0) {
            i++;
            if (i == argc) {
                fprintf(stderr, "Sequence data file name missing.\n");
                return 0;
            }
            check_file(argv[i], "r");
            config.sequence_file = argv[i];
        } else if (strcmp(argv[i], "-k") == 0 || strcmp(argv[i], "--ksize") == 0) {
            i++;
            if (i == argc) {
                fprintf(stderr, "Number for size of k is missing.\n");
                return 0;
            } else {
                int k = atoi(argv[i]);
                if (k < 0 || k > 20) {
                    fprintf(stderr,
                            "%d is not a valid value for k.\nPlease select a number greater than zero and less than 21\n",
                            k);
                    exit(EXIT_FAILURE);
                }
                config.k = k;
            }
        } else if (strcmp(argv[i], "-q") == 0 || strcmp(argv[i], "--quiet") == 0) {
            i++;
            if (i == argc) {
                fprintf(stderr,
                        "True/false value for quiet option is missing.\nUsage is \"-q 1\" for suppression OR \"-q 0\" for expansion\n");
                exit(EXIT_FAILURE);
            } else {
                int opt = atoi(argv[i]);
                if (opt == 1 || opt == 0) {
                    config.suppressOutputEnable = opt;
                } else {
                    fprintf(stderr,
                            "%d is not a valid value for suppress Output Enable Option.\nPlease select either 0 for FALSE or a 1 for TRUE",
                            opt);
                    exit(EXIT_FAILURE);
                }
            }
        } else if (strcmp(argv[i], "-z") == 0 || strcmp(argv[i], "--zthreshold") == 0) {
            i++;
            if (i == argc) {
                fprintf(stderr, "Z threshold number is missing\nUsage is \"-z 1000\".\n");
                exit(EXIT_FAILURE);
            } else {
                config.zThresholdEnable = 1;
                config.zThreshold = atoi(argv[i]);
            }
        } else if (strcmp(argv[i], "--sweep") == 0) {
            i++;
            if (i == argc) {
                fprintf(stderr, "Largest k for --sweep is missing.\nUsage is \"-k 6 --sweep 11\".\n");
                exit(EXIT_FAILURE);
            }
            sweep_kmax = atoi(argv[i]);
        } else {
            fprintf(stderr, "Ignoring invalid option %s\n", argv[i]);
            if (config.suppressOutputEnable == 0) {
                fprintf(stderr, "Press enter to continue.\n");
                getchar();
            }
        }
        i++;
    }
    return 1;
}

static unsigned long estimate_RAM_usage() {                         /* :1226-1291 */
    const unsigned long node_t_size = 48;   /* sizeof(node_t) on x86-64 (:107-111) */
    unsigned long maxNumberOfNodes = 1;
    double n = 1;
    while (n <= config.k) maxNumberOfNodes += pow(4.0, n++);
    if (((sizeof(char) * (config.k + 10)) * maxNumberOfNodes) >= (1024 * 1024 * 1024)) {
        std::cout << ((sizeof(char) * (config.k + 10)) * maxNumberOfNodes) / (double)(1024 * 1024 * 1024)
                  << " gibibytes";
    } else {
        std::cout << ((sizeof(char) * (config.k + 10)) * maxNumberOfNodes) / (double)(1024 * 1024)
                  << " mibibytes";
    }
    std::cout << " of disk usage and ";
    if (maxNumberOfNodes * node_t_size >= (1024 * 1024 * 1024)) {
        std::cout << (maxNumberOfNodes * node_t_size / (double)(1024 * 1024 * 1024))
                  << " gibibytes of RAM usage likely" << std::endl;
        std::cout << "We are stopping here to make sure that is ok with you!" << std::endl;
        std::cout << "Hit enter to proceed or else abort the program." << std::endl;
        if (config.suppressOutputEnable == 0) getchar();
    } else {
        std::cout << (maxNumberOfNodes * node_t_size / (double)(1024 * 1024))
                  << " mibibytes of RAM usage likely" << std::endl;
    }
    return maxNumberOfNodes;
}

static void die_engine(int rc) {
    fprintf(stderr, "findKmer: GPU engine error: %s\n", fk_strerror(rc));
    exit(EXIT_FAILURE);
}

/* "Unknown character" warnings (:582-584) of the unknown bytes not yet
   printed, in stream order; by_pos: only those before stream offset `limit`
   (the engine collects their offsets, collect_unknown = 2).  The reference
   prints them during its scan, between the -q 0 progress lines (:997). */
static uint64_t g_unk_done = 0;
static void flush_unknown(fk_engine *e, uint64_t limit, bool by_pos) {
    uint64_t n = 0;
    if (fk_engine_unknown_since(e, g_unk_done, nullptr, nullptr, 0, &n)) return;
    std::vector<uint8_t> u;
    std::vector<uint64_t> p;
    while (g_unk_done < n) {
        const uint64_t m = std::min<uint64_t>(n - g_unk_done, 1u << 16);
        u.resize((size_t)m);
        p.resize(by_pos ? (size_t)m : 0);
        if (fk_engine_unknown_since(e, g_unk_done, u.data(), by_pos ? p.data() : nullptr, m, &n)) return;
        for (uint64_t i = 0; i < m; i++) {
            if (by_pos && p[(size_t)i] >= limit) return;
            fprintf(stderr, "Unknown character %c processed! File may be corrupted.\n", (char)u[(size_t)i]);
            g_unk_done++;
        }
    }
}

/*
 * Drive the engine over the whole file.  With quiet == 0 the reference prints
 * "Read %llu bases\n>" + the header line at every '>' that starts a comment
 * (:996-1002), with baseCounter as of that point; we feed the engine up to
 * each such '>' and read its running counter (host only splits the stream).
 */
static int scan_file(fk_engine *e, FILE *f, fk_result *res, bool echo = true) {
    const size_t PIECE = 256u << 20;
    std::vector<uint8_t> buf(PIECE);
    int in_hdr = 0, ended = 0;
    for (;;) {
        size_t n = fread(buf.data(), 1, buf.size(), f);
        if (n == 0) break;
        if (config.suppressOutputEnable != 0 || !echo || ended) {
            int rc = fk_engine_feed(e, buf.data(), n, 0);
            if (rc) return rc;
            continue;
        }
        size_t pos = 0;
        while (pos < n) {
            int rc;
            if (ended) {
                rc = fk_engine_feed(e, buf.data() + pos, n - pos, 0);
                if (rc) return rc;
                break;
            }
            if (in_hdr) {                        /* echo the header line (:999-1002) */
                size_t r = pos;
                while (r < n && buf[r] != '\n') fputc(buf[r++], stdout);
                rc = fk_engine_feed(e, buf.data() + pos, r - pos, 0);
                if (rc) return rc;
                if (r == n) break;               /* continues in the next piece */
                fprintf(stdout, "\n");
                rc = fk_engine_feed(e, buf.data() + r, 1, 0);
                if (rc) return rc;
                in_hdr = 0;
                pos = r + 1;
                continue;
            }
            size_t q = pos;
            while (q < n && buf[q] != '>' && buf[q] != 0xFF) q++;
            if (q > pos) {
                rc = fk_engine_feed(e, buf.data() + pos, q - pos, 0);
                if (rc) return rc;
            }
            if (q == n) break;
            if (buf[q] == 0xFF) {                /* (char)0xFF == EOF ends the scan (:988) */
                ended = 1;
                pos = q;
                continue;
            }
            uint64_t vb = 0;
            rc = fk_engine_progress(e, &vb, nullptr);
            if (rc) return rc;
            flush_unknown(e, 0, false);   /* the warnings of the bytes before this '>' */
            fprintf(stdout, "Read %llu bases\n%c", (unsigned long long)vb, '>');   /* :997 */
            rc = fk_engine_feed(e, buf.data() + q, 1, 0);
            if (rc) return rc;
            in_hdr = 1;
            pos = q + 1;
        }
    }
    return fk_engine_finish(e, res);
}

/* -q 0 on a device-resident file: the progress lines of every comment line
   (:996-1002) come from fk_input_headers (load_headers; FK_E_STATE when the
   file needs the streamed path), the header text from the file; after the
   scan, the unknown-character warnings go between them in stream order. */
static int load_headers(int k, std::vector<uint64_t> &pos, std::vector<uint64_t> &bases) {
    uint64_t n = 0;
    int rc = fk_input_headers(g_input, k, nullptr, nullptr, 0, &n);
    if (rc) return rc;
    pos.assign((size_t)n + 1, 0);
    bases.assign((size_t)n + 1, 0);
    rc = fk_input_headers(g_input, k, pos.data(), bases.data(), n, &n);
    pos.resize((size_t)n);
    bases.resize((size_t)n);
    return rc;
}

static int print_progress(fk_engine *eng, const std::vector<uint64_t> &pos, const std::vector<uint64_t> &bases) {
    const uint64_t n = pos.size();
    /* the header text from a read-only mapping of the file */
    const int fd = fileno(config.sequence_file_pointer);
    struct stat sb;
    if (fstat(fd, &sb) != 0) return FK_E_IO;
    const size_t size = (size_t)sb.st_size;
    const uint8_t *m = nullptr;
    if (size) {
        void *p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (p == MAP_FAILED) return FK_E_IO;
        madvise(p, size, MADV_SEQUENTIAL);
        m = static_cast<const uint8_t *>(p);
    }
    for (uint64_t i = 0; i < n; i++) {
        flush_unknown(eng, pos[(size_t)i], true);
        fprintf(stdout, "Read %llu bases\n%c", (unsigned long long)bases[(size_t)i], '>');   /* :997 */
        const size_t b = (size_t)pos[(size_t)i] + 1;
        const uint8_t *e = b < size ? static_cast<const uint8_t *>(memchr(m + b, '\n', size - b)) : nullptr;
        const size_t end = e ? (size_t)(e - m) : size;
        if (end > b) fwrite(m + b, 1, end - b, stdout);       /* echo the line (:999-1002) */
        if (e) fputc('\n', stdout);
    }
    if (m) munmap(const_cast<uint8_t *>(m), size);
    return FK_OK;
}

/* The whole file, device-resident (fk_input_load), in one feed. */
static int scan_device(fk_engine *e, fk_result *res) {
    const uint8_t *d = nullptr;
    uint64_t len = 0;
    int rc = fk_input_info(g_input, &d, &len, nullptr, nullptr);
    if (rc) return rc;
    rc = fk_engine_feed(e, d, len, 1);
    if (rc) return rc;
    return fk_engine_finish(e, res);
}

/* One k: the reference's main() from print_conf() on (:1303-1379). */
static int run_k(int argc) {
    print_conf(argc);
    unsigned long maxNumberOfNodes = estimate_RAM_usage();
    (void)maxNumberOfNodes;

    fprintf(stdout, "!!!Find The KMER!!!\n");
    fprintf(stdout, "Reading sequence from file\n");
    fprintf(stdout, "     2858658142 bases in the reference genome FYI.\nThat is 2,858,658,142 by the way.\n");
    /* (no flush here: the reference's stdout stays buffered through its scan,
       and its "Unknown character" warnings (stderr) land between the
       buffered blocks exactly where ours do -- the same bytes, flushed at
       the same points) */

    /* empty-file check (:982-985) */
    int c0 = fgetc(config.sequence_file_pointer);
    if (c0 == EOF) {
        fprintf(stderr, "Sequence File Is Empty, Ending Program");
        exit(EXIT_FAILURE);
    }
    rewind(config.sequence_file_pointer);

    double tp = now_s();
    if (g_times && !g_input_tried) {
        fk_device_count();   /* the HIP runtime's start-up, timed on its own */
        phase(config.k, "hip_init", tp);
    }
    /* load the file to HBM once (and reuse it for every k of a sweep) */
    if (!g_input_tried) {
        g_input_tried = true;
        /* the GPU of this process (fk_device_select: FINDKMER_DEVICE, else
           spread over the devices with room for the file and the engine's
           buffers: ~2 bytes of partition codes per input byte for
           8 <= k <= 13; for k >= 17 the engine keeps a copy of the input
           for its key-range passes, whose scratch fits what is left) */
        struct stat sb;
        const uint64_t fsize = stat(config.sequence_file, &sb) == 0 ? (uint64_t)sb.st_size : 0;
        const int kk = sweep_kmax > config.k ? sweep_kmax : config.k;
        /* bytes per input byte: the file + partition codes (16-bit: 2 per
           region; 32-bit for k = 15, 16: 8, + 2 of part streams), or for
           k >= 17 the engine's copy of the input; plus the dense table (and
           for 8 <= k <= 12 the 4^(k+1) pair + 4^k single bins of pairs mode) */
        const uint64_t per = kk > FK_K_MAX_DENSE ? 3 : kk >= 15 ? 11 : (kk >= 8 ? 4 : 2);
        const uint64_t table = kk > FK_K_MAX_DENSE ? 0 : (4ull << (2 * kk)) * (kk >= 8 && kk <= 12 ? 6 : 1);   /* + pair bins */
        int dsel = fk_device_select(fsize * per + table + (256ull << 20), &g_device);
        if (dsel == FK_E_INVALID) {
            fprintf(stderr, "findKmer: FINDKMER_DEVICE names no visible GPU\n");
            exit(EXIT_FAILURE);
        }
        if (dsel) die_engine(dsel);
        const char *ing = getenv("FINDKMER_INGEST");
        if (!ing || strcmp(ing, "stream") != 0) {
            const char *nt = getenv("FINDKMER_INGEST_THREADS");   /* default: the library's choice */
            int lrc = fk_input_load(config.sequence_file, g_device, nt ? atoi(nt) : 0, &g_input);
            if (lrc == FK_E_HIP || lrc == FK_E_NO_DEVICE) die_engine(lrc);
            /* not a regular file, or larger than free HBM: stream it */
            if (lrc) g_input = nullptr;
        }
    }
    phase(config.k, "ingest", tp);
    bool on_device = g_input != nullptr;
    /* -q 0: the per-record progress lines, from the device copy */
    bool progress = on_device && config.suppressOutputEnable == 0;
    std::vector<uint64_t> hpos, hbases;
    if (progress) {
        int prc = load_headers(config.k, hpos, hbases);
        if (prc == FK_E_STATE) on_device = progress = false;   /* 0xFF / int32 zone: the streamed path prints them */
        else if (prc) die_engine(prc);
    }
    g_unk_done = 0;

    fk_opts opts;
    memset(&opts, 0, sizeof opts);
    opts.device = g_device;
    if (on_device) fk_input_info(g_input, nullptr, nullptr, &opts.device, nullptr);
    opts.want_nodes = 1;
    opts.collect_unknown = progress ? 2 : 1;   /* 2: with their offsets, to interleave */
    /* k >= 17: finish re-reads the resident file, which outlives the engine,
       instead of keeping a copy of it */
    opts.borrow_input = on_device ? 1 : 0;
    fk_engine *eng = nullptr;
    int rc = fk_engine_create(config.k, &opts, &eng);
    if (rc) die_engine(rc);
    phase(config.k, "engine_create", tp);
    fk_result res;
    rc = on_device ? scan_device(eng, &res) : scan_file(eng, config.sequence_file_pointer, &res);
    phase(config.k, "scan", tp);
    if (rc == FK_E_OOM && on_device) {
        /* the resident file copy and the engine's buffers (k >= 17: its own
           copy of the input plus a pass's scratch) do not fit together: drop
           the file copy and stream the file through the engine's pinned
           staging instead */
        fk_input_destroy(g_input);
        g_input = nullptr;
        rc = fk_engine_reset(eng);
        if (rc) die_engine(rc);
        rewind(config.sequence_file_pointer);
        rc = scan_file(eng, config.sequence_file_pointer, &res);
        progress = false;   /* the streamed path printed them */
    }
    if (progress && (rc == FK_OK || rc == FK_E_ROLLOVER || rc == FK_E_UNTERMINATED_HEADER)) {
        const int prc = print_progress(eng, hpos, hbases);
        if (prc) die_engine(prc);
    }
    /* the "Unknown character" warnings not printed yet (:582-584): after the
       last progress line, in stream order */
    flush_unknown(eng, 0, false);
    if (rc == FK_E_ROLLOVER) {                                       /* :642-648 */
        const char *m = "\n\n!!! COUNTER ROLLOVER DETECTED! \nIncrease the number of bits used for the counter variable if you have the source code, else use a smaller sequence file.\n\n";
        fprintf(stderr, "%s", m);
        fprintf(stdout, "%s", m);
        exit(EXIT_FAILURE);
    }
    if (rc == FK_E_UNTERMINATED_HEADER) {
        fprintf(stderr, "findKmer: the sequence file ends inside a '>' header line (the reference program hangs here)\n");
        exit(EXIT_FAILURE);
    }
    if (rc != FK_OK && rc != FK_E_EMPTY) die_engine(rc);

    std::string stats_name = std::to_string(config.k) + "mer_Base_Stats_Of_" + config.sequence_file + ".txt";
    double prob[4];
    int st = fk_write_stats(stats_name.c_str(), config.k, &res, stdout, prob);
    if (st == 1 || st == FK_E_IO) {
        fflush(config.out_file_pointer);
        exit(EXIT_FAILURE);
    }

    phase(config.k, "stats", tp);
    fprintf(stdout, "Now creating histogram.\n");
    fflush(stdout);
    if (config.k > FK_K_MAX_DENSE) {
        /* 17 <= k <= 20: the engine's sparse table (distinct k-mers, sorted) */
        uint64_t n = 0;
        rc = fk_engine_sparse(eng, nullptr, nullptr, 0, &n);
        if (rc) die_engine(rc);
        std::vector<uint64_t> keys((size_t)n + 1);
        std::vector<uint32_t> cnts((size_t)n + 1);
        rc = fk_engine_sparse(eng, keys.data(), cnts.data(), n, &n);
        if (rc) die_engine(rc);
        fk_engine_destroy(eng);
        rc = fk_write_rows_sparse(config.out_file_pointer, config.k, keys.data(), cnts.data(), n, prob, res.windows,
                                  config.zThresholdEnable, (double)config.zThreshold, 0);
    } else {
        std::vector<uint32_t> counts((size_t)1 << (2 * config.k));
        rc = fk_engine_table(eng, counts.data());
        if (rc) die_engine(rc);
        fk_engine_destroy(eng);
        phase(config.k, "table_copy", tp);
        rc = fk_write_rows(config.out_file_pointer, config.k, counts.data(), prob, res.windows,
                           config.zThresholdEnable, (double)config.zThreshold, 0);
    }
    if (rc) die_engine(rc);
    phase(config.k, "histogram", tp);

    fprintf(stdout, "histogram creation finished.\n");
    if (fclose(config.out_file_pointer) == EOF) {
        fprintf(stderr,
                "Out file close error! This is not expected and might mean the data was not written to the file properly before the close.\n");
    }
    fprintf(stdout, "Your file can be found in the current directory as: \n    %s\n", config.out_file.c_str());
    if (fclose(config.sequence_file_pointer) == EOF) {
        fprintf(stderr, "Sequence file close error! This is likely ok though.\n");
    }
    return 0;
}

int main(int argc, char *argv[]) {                                  /* :1292-1379 */
    const char *tm = getenv("FINDKMER_TIMES");
    g_times = tm && tm[0] == '1';
    double t_main = now_s();
    init_conf();
    usage();
    if (!parse_arguments(argc, argv)) {
        usage();
        return EXIT_FAILURE;
    }
    const bool explicit_out = config.out_set;
    const int kfirst = config.k ? config.k : DEFAULT_K_VALUE;
    int klast = kfirst;
    if (sweep_kmax >= 0) {
        if (explicit_out || sweep_kmax < kfirst || sweep_kmax > 20) {
            fprintf(stderr, "--sweep %d: needs %d <= KMAX <= 20 and no -e (one output file per k)\n", sweep_kmax,
                    kfirst);
            return EXIT_FAILURE;
        }
        klast = sweep_kmax;
    }
    int rc = 0;
    for (int k = kfirst; k <= klast && rc == 0; k++) {
        config.k = k;
        if (!explicit_out) config.out_set = false;
        if (k > kfirst) usage();   /* stdout == the separate runs' stdout, concatenated */
        rc = run_k(argc);
    }
    if (g_input) fk_input_destroy(g_input);
    phase(config.k, "main_total", t_main);
    /* every output is written and closed, and the device work is complete:
       leave without the HIP runtime's teardown (tens of ms per run of the
       sweep script's six) */
    fflush(stdout);
    fflush(stderr);
    _exit(rc);
}
