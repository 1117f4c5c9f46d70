// cli.cpp -- `rustseq_mini`, the reference CLI (smith_waterman/src/main.rs)
// rebuilt over the MI355X scorer's C ABI (include/msw.h, include/msw_fastq.h).
//
// Flags of main.rs:11-46 are kept (-1/--seq1, -2/--seq2, -f/--files,
// -c/--chunk-size (unused, as in the reference), -g/--gpu, -n/--num-files
// (unused), -t/--test-wgs, --full-wgs), plus:
//   --score-mode compat|sw   compat (default) = the kernel the reference launches
//                            (smith_waterman.cl:11-71); sw = Smith-Waterman
//   --gap-model linear|affine, --match/--mismatch/--gap-open/--gap-extend
//   --reference FASTA        sw --full-wgs: read i is scored against
//                            reference[pos : pos + window], pos from the
//                            "pos=" tag of its FASTQ header
//   --window N               window length (default 2 x read length)
//   --num-gpus N             --full-wgs: lane files sharded over N GPUs
//   --checkpoint-dir DIR     checkpoint_<run_id>.json written per file, resumed
//   --json PATH              run record (benchmark.rs:17-34 fields + GCUPS)
// Environment (.env loaded like dotenv, main.rs:50): WGS_DATA_DIR,
// WGS_SAMPLE_ID, WGS_LANES, WGS_READS_PER_LANE (aligner.rs:184-195),
// GPU_CHUNK_SIZE_READS (mandatory for chunked modes, aligner.rs:9-15),
// WGS_RUN_ID (stable checkpoint id).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <ctime>
#include <vector>

#include "msw.h"
#include "msw_fastq.h"

namespace {

using Clock = std::chrono::steady_clock;

double ms_since(Clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

// Exit 1 with a message.  _exit: a worker thread may die while others are
// still inside HIP calls, and exit()'s static destructors (the HIP runtime's
// teardown) would race them.
[[noreturn]] void die(const std::string& msg) {
    fflush(stdout);
    fprintf(stderr, "%s\n", msg.c_str());
    fflush(stderr);
    _exit(1);
}

std::string env_or(const char* k, const std::string& d) {
    const char* v = getenv(k);
    return v ? std::string(v) : d;
}

// dotenv::dotenv().ok() (main.rs:50): KEY=VALUE lines of ./.env, existing
// variables win, missing file is fine.
void load_dotenv() {
    std::ifstream f(".env");
    std::string line;
    while (std::getline(f, line)) {
        if (line.empty() || line[0] == '#') continue;
        const size_t eq = line.find('=');
        if (eq == std::string::npos) continue;
        std::string k = line.substr(0, eq), v = line.substr(eq + 1);
        while (!k.empty() && isspace((unsigned char)k.back())) k.pop_back();
        while (!v.empty() && isspace((unsigned char)v.front())) v.erase(v.begin());
        if (v.size() >= 2 && (v.front() == '"' || v.front() == '\'') && v.back() == v.front())
            v = v.substr(1, v.size() - 2);
        setenv(k.c_str(), v.c_str(), 0);
    }
}

// CPUs this process may use: the affinity mask, capped by the cgroup v2 CPU
// quota (cpu.max) when there is one.  The GPU boxes grant a 16-CPU quota on a
// 256-CPU affinity mask, so hardware_concurrency() alone overstates it 16x.
int usable_cpus() {
    int n = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[64] = {0};
        double period = 0;
        if (fscanf(f, "%63s %lf", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
            const int quota = (int)(atof(q) / period);
            if (quota >= 1) n = std::min(n, quota);
        }
        fclose(f);
    }
    return std::max(1, n);
}

// aligner.rs:9-15
uint64_t get_chunk_size_reads() {
    const char* v = getenv("GPU_CHUNK_SIZE_READS");
    if (!v) die("error: GPU_CHUNK_SIZE_READS not set in .env file");
    char* end = nullptr;
    unsigned long long n = strtoull(v, &end, 10);
    if (!*v || *end || n == 0) die(std::string("error: Invalid GPU_CHUNK_SIZE_READS value '") + v + "'");
    return n;
}

struct Args {
    std::string seq1, seq2;
    bool has_seq1 = false, has_seq2 = false, files = false, gpu = false, test_wgs = false, full_wgs = false;
    long chunk_size = 1, num_files = -1;
    std::string score_mode = "compat", gap_model = "linear", reference, checkpoint_dir = ".", json, scores_out;
    int match = 2, mismatch = -1, gap_open = 3, gap_extend = -1, window = 0, num_gpus = 1;
};

void usage() {
    printf(
        "High-performance sequence alignment for genome-scale data (MI355X)\n\n"
        "Usage: rustseq_mini [OPTIONS]\n\n"
        "Options:\n"
        "  -1, --seq1 <SEQ1>            first sequence or file path\n"
        "  -2, --seq2 <SEQ2>            second sequence or file path\n"
        "  -f, --files                  treat inputs as file paths instead of direct sequences\n"
        "  -c, --chunk-size <N>         chunk size in MB (accepted, unused as in the reference)\n"
        "  -g, --gpu                    use GPU acceleration if available\n"
        "  -n, --num-files <N>          number of files (accepted, unused as in the reference)\n"
        "  -t, --test-wgs               count bases of the first lane's files\n"
        "      --full-wgs               process the full WGS dataset\n"
        "      --score-mode <compat|sw> compat = reference kernel semantics (default), sw = Smith-Waterman\n"
        "      --gap-model <linear|affine>\n"
        "      --match N --mismatch N --gap-open N --gap-extend N\n"
        "      --reference <FASTA>      reference genome for --full-wgs --score-mode sw\n"
        "      --window N               window length (default 2 x read length)\n"
        "      --num-gpus N             GPUs for --full-wgs\n"
        "      --checkpoint-dir DIR     where checkpoint_<run_id>.json lives (default .)\n"
        "      --scores-out DIR         --full-wgs sw: per-read results, one <lane file>.scores per file\n"
        "                               (8 bytes per read in file order: i32 score, i16 end_i, i16 end_j)\n"
        "      --json PATH              write a JSON run record\n"
        "  -h, --help\n");
}

Args parse_args(int argc, char** argv) {
    Args a;
    auto need = [&](int& i) -> std::string {
        if (i + 1 >= argc) die(std::string("error: a value is required for '") + argv[i] + "'");
        return argv[++i];
    };
    for (int i = 1; i < argc; ++i) {
        std::string s = argv[i];
        std::string val;
        const size_t eq = s.find('=');
        if (s.rfind("--", 0) == 0 && eq != std::string::npos) { val = s.substr(eq + 1); s = s.substr(0, eq); }
        auto v = [&]() { return val.empty() ? need(i) : val; };
        if (s == "-1" || s == "--seq1") { a.seq1 = v(); a.has_seq1 = true; }
        else if (s == "-2" || s == "--seq2") { a.seq2 = v(); a.has_seq2 = true; }
        else if (s == "-f" || s == "--files") a.files = true;
        else if (s == "-c" || s == "--chunk-size") a.chunk_size = atol(v().c_str());
        else if (s == "-g" || s == "--gpu") a.gpu = true;
        else if (s == "-n" || s == "--num-files") a.num_files = atol(v().c_str());
        else if (s == "-t" || s == "--test-wgs") a.test_wgs = true;
        else if (s == "--full-wgs") a.full_wgs = true;
        else if (s == "--score-mode") a.score_mode = v();
        else if (s == "--gap-model") a.gap_model = v();
        else if (s == "--match") a.match = atoi(v().c_str());
        else if (s == "--mismatch") a.mismatch = atoi(v().c_str());
        else if (s == "--gap-open") a.gap_open = atoi(v().c_str());
        else if (s == "--gap-extend") a.gap_extend = atoi(v().c_str());
        else if (s == "--reference") a.reference = v();
        else if (s == "--window") a.window = atoi(v().c_str());
        else if (s == "--num-gpus") a.num_gpus = atoi(v().c_str());
        else if (s == "--checkpoint-dir") a.checkpoint_dir = v();
        else if (s == "--json") a.json = v();
        else if (s == "--scores-out") a.scores_out = v();
        else if (s == "-h" || s == "--help") { usage(); exit(0); }
        else die("error: unexpected argument '" + s + "' found\n\nFor more information, try '--help'.");
    }
    if (a.score_mode != "compat" && a.score_mode != "sw") die("error: --score-mode must be compat or sw");
    if (a.gap_model != "linear" && a.gap_model != "affine") die("error: --gap-model must be linear or affine");
    if (a.gap_extend < 0) a.gap_extend = a.gap_model == "affine" ? 1 : 2;
    return a;
}

// Best cells cost ~1.5x the score-only kernel; --full-wgs needs them only for
// --scores-out records (the per-file results are score sums), pair mode prints
// them.
msw_scoring_t scoring_of(const Args& a, bool want_coords) {
    msw_scoring_t sc;
    sc.match = a.match;
    sc.mismatch = a.mismatch;
    sc.gap_open = a.gap_model == "affine" ? a.gap_open : 0;
    sc.gap_extend = a.gap_extend;
    sc.affine = a.gap_model == "affine";
    sc.want_coords = want_coords ? 1 : 0;
    return sc;
}

struct Device {
    int ordinal;
    std::string name;
    double memory_gb;
    uint32_t max_wg;
};

bool is_gpu_available() {
    int n = 0;
    return msw_device_count(&n) == MSW_OK && n > 0;
}

std::vector<Device> get_gpu_devices() {
    std::vector<Device> out;
    int n = 0;
    if (msw_device_count(&n) != MSW_OK) return out;
    for (int i = 0; i < n; ++i) {
        msw_device_info_t info;
        if (msw_device_info(i, &info) != MSW_OK) continue;
        out.push_back({i, info.name, info.mem_bytes / 1073741824.0, info.max_wg});
    }
    return out;
}

struct Ctx {
    msw_ctx* h = nullptr;
    // --full-wgs workers leave their context (and buffers) to the process
    // exit: main ends the process with _exit once the run record and the
    // checkpoint are written, so releasing them one by one (50-60 ms of
    // unregisters and frees after the last results) is work the OS redoes
    bool keep = false;
    explicit Ctx(int ordinal, unsigned flags = 0) {
        if (msw_ctx_create_ex(ordinal, flags, &h) != MSW_OK) die(std::string("GPU context error: ") + msw_last_error());
    }
    ~Ctx() {
        if (!keep) msw_ctx_destroy(h);
    }
};

// gpu_align (aligner.rs:410-532) through msw_align_compat.
int32_t gpu_align(Ctx& ctx, const std::string& s1, const std::string& s2, const Device& dev, bool* ok,
                  std::string* err) {
    int32_t score = 0;
    const uint32_t wg = std::min<uint32_t>(dev.max_wg, 1024);
    const int rc = msw_align_compat(ctx.h, (const uint8_t*)s1.data(), s1.size(), (const uint8_t*)s2.data(),
                                    s2.size(), wg, 1000000, &score);
    *ok = rc == MSW_OK;
    if (!*ok && err) *err = msw_last_error();
    return score;
}

// A FASTQ file as chunks of concatenated sequences (the Vec<String> + concat
// of aligner.rs:270 / :392-393).
int for_each_fastq_chunk(const std::string& path, uint64_t chunk, const std::function<int(std::string&)>& fn,
                         uint64_t* bases = nullptr, uint64_t* reads = nullptr) {
    msw_fastq* fq = nullptr;
    if (msw_fastq_open(path.c_str(), &fq) != MSW_OK) return -1;
    constexpr uint32_t kStride = 4096;
    std::vector<uint8_t> slab((size_t)std::min<uint64_t>(chunk, 65536) * kStride);
    std::vector<uint16_t> lens(std::min<uint64_t>(chunk, 65536));
    std::string cat;
    uint64_t in_chunk = 0, nb = 0, nr = 0;
    int rc = 0;
    for (;;) {
        uint64_t want = std::min<uint64_t>(chunk - in_chunk, lens.size()), got = 0;
        rc = msw_fastq_next(fq, slab.data(), lens.data(), kStride, want, &got, nullptr);
        if (rc) break;
        for (uint64_t i = 0; i < got; ++i) {
            cat.append((const char*)slab.data() + i * kStride, lens[i]);
            nb += lens[i];
        }
        nr += got;
        in_chunk += got;
        if (got == 0 || in_chunk == chunk) {
            if (in_chunk > 0) {
                rc = fn(cat);
                if (rc) break;
            }
            cat.clear();
            in_chunk = 0;
            if (got == 0) break;
        }
    }
    msw_fastq_close(fq);
    if (bases) *bases = nb;
    if (reads) *reads = nr;
    return rc;
}

// ---------------------------------------------------------------------------
// Reference genome (FASTA) for sw mode.
// ---------------------------------------------------------------------------
// The sequence lines concatenated (header lines and '\r' dropped): the file is
// mapped and scanned with memchr (about 2x the line-by-line rate).  Returns
// false when the file cannot be read.
bool load_fasta(const std::string& path, std::string* seq) {
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    struct stat sb;
    if (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode)) {
        close(fd);
        return false;
    }
    seq->clear();
    const size_t n = (size_t)sb.st_size;
    void* m = n ? mmap(nullptr, n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0) : nullptr;
    close(fd);
    if (n && m == MAP_FAILED) return false;
    seq->reserve(n);
    const char* p = (const char*)m;
    const char* end = p + n;
    while (p < end) {
        const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
        const char* e = nl ? nl : end;
        const char* le = (e > p && e[-1] == '\r') ? e - 1 : e;
        if (le > p && *p != '>') seq->append(p, (size_t)(le - p));
        p = e + 1;
    }
    if (n) munmap(m, n);
    return true;
}

// The reference, loaded on a thread of its own from the start of main, beside
// the HIP runtime init; run_full_wgs takes it before the workers start.
struct ReferenceLoad {
    std::string path, seq;
    double ms = 0;
    bool ok = false;
    std::thread th;
    void start(const std::string& p) {
        path = p;
        th = std::thread([this]() {
            const auto t = Clock::now();
            ok = load_fasta(path, &seq);
            ms = ms_since(t);
        });
    }
    // the sequence; exits like the other setup errors when it could not be read
    const std::string& get() {
        std::call_once(joined, [this]() {
            if (th.joinable()) th.join();
        });
        if (!ok) die("error: cannot open reference " + path);
        return seq;
    }
    ~ReferenceLoad() {
        if (th.joinable()) th.join();
    }
    std::once_flag joined;
};

// ---------------------------------------------------------------------------
// Checkpoint / resume (aligner.rs:22-104 schema, with the bugs fixed: one
// stable file name per run id, i64 scores, resume skips completed files).
// ---------------------------------------------------------------------------
struct FileCheckpoint {
    std::string file_path;
    size_t file_index = 0;
    long long score = 0;
    double processing_time_ms = 0;
    unsigned long long total_bases = 0, total_reads = 0;
    bool completed = false;
};

std::string json_escape(const std::string& s) {
    std::string o;
    for (char c : s) {
        if (c == '"' || c == '\\') { o += '\\'; o += c; }
        else if ((unsigned char)c < 0x20) { char b[8]; snprintf(b, sizeof(b), "\\u%04x", c); o += b; }
        else o += c;
    }
    return o;
}

struct Checkpoint {
    std::string run_id, path;
    size_t total_files = 0;
    std::map<size_t, FileCheckpoint> files;

    void save() const {
        std::ostringstream o;
        size_t done = 0;
        for (auto& kv : files) done += kv.second.completed;
        o << "{\n  \"run_id\": \"" << json_escape(run_id) << "\",\n  \"files\": [";
        bool first = true;
        for (auto& kv : files) {
            const FileCheckpoint& f = kv.second;
            o << (first ? "\n" : ",\n") << "    {\"file_path\": \"" << json_escape(f.file_path)
              << "\", \"file_index\": " << f.file_index << ", \"score\": " << f.score
              << ", \"processing_time_ms\": " << f.processing_time_ms << ", \"total_bases\": " << f.total_bases
              << ", \"total_reads\": " << f.total_reads << ", \"completed\": " << (f.completed ? "true" : "false")
              << "}";
            first = false;
        }
        o << "\n  ],\n  \"total_files\": " << total_files << ",\n  \"completed_files\": " << done << "\n}\n";
        const std::string tmp = path + ".tmp";
        {
            std::ofstream f(tmp);
            f << o.str();
        }
        rename(tmp.c_str(), path.c_str());  // atomic replace
    }

    // Minimal parser for the file this program writes.
    bool load() {
        std::ifstream f(path);
        if (!f) return false;
        std::stringstream ss;
        ss << f.rdbuf();
        const std::string s = ss.str();
        size_t p = 0;
        while ((p = s.find("{\"file_path\": \"", p)) != std::string::npos) {
            FileCheckpoint c;
            size_t q = s.find('"', p + 15);
            c.file_path = s.substr(p + 15, q - (p + 15));
            auto num = [&](const char* key) -> std::string {
                size_t k = s.find(key, q);
                if (k == std::string::npos) return "0";
                k += strlen(key);
                size_t e = s.find_first_of(",}", k);
                return s.substr(k, e - k);
            };
            c.file_index = strtoull(num("\"file_index\": ").c_str(), nullptr, 10);
            c.score = strtoll(num("\"score\": ").c_str(), nullptr, 10);
            c.processing_time_ms = atof(num("\"processing_time_ms\": ").c_str());
            c.total_bases = strtoull(num("\"total_bases\": ").c_str(), nullptr, 10);
            c.total_reads = strtoull(num("\"total_reads\": ").c_str(), nullptr, 10);
            c.completed = num("\"completed\": ").find("true") != std::string::npos;
            files[c.file_index] = c;
            p = q;
        }
        return true;
    }
};

// ---------------------------------------------------------------------------
// --full-wgs driver: reader threads fill read slabs, a bounded queue hands
// chunks to one host thread per GPU (own msw_ctx), results are summed per file.
// ---------------------------------------------------------------------------
// Read slab stride of sw mode: MSW_MAX_READ_LEN (default 256, the packed
// kernels' read limit; up to 32767 -- longer reads then score on the
// long-pair kernel, with either lane reader).
// (read on first use, so a bad value fails the run that needs it, not --help)
uint32_t read_stride() {
    static const uint32_t stride = [] {
        const long v = atol(env_or("MSW_MAX_READ_LEN", "256").c_str());
        if (v < 1 || v > 32767) die("error: MSW_MAX_READ_LEN must be in [1, 32767]");
        return std::max<uint32_t>(16u, ((uint32_t)v + 15u) & ~15u);
    }();
    return stride;
}

// Read slabs in pinned memory (msw_host_alloc = hipHostMalloc): the FASTQ
// readers parse straight into them and msw_align_reads DMAs them to the GPU
// without staging.  Recycled through a free list; one block per slab:
// [reads cap x read_stride() | pos i64 x cap | rlen u16 x cap].
class SlabPool {
   public:
    struct Slab {
        uint8_t* base = nullptr;
        uint8_t* reads = nullptr;
        int64_t* pos = nullptr;
        uint16_t* rlen = nullptr;
        bool pinned = false;
    };
    explicit SlabPool(uint64_t cap) : cap_(cap) {}
    ~SlabPool() {
        for (Slab* s : free_) release(s);
    }
    Slab* get() {
        {
            std::lock_guard<std::mutex> lk(m_);
            if (!free_.empty()) {
                Slab* s = free_.back();
                free_.pop_back();
                return s;
            }
        }
        Slab* s = new Slab();
        const size_t bytes = cap_ * (read_stride() + 8 + 2);
        s->base = (uint8_t*)msw_host_alloc(bytes);
        s->pinned = s->base != nullptr;
        if (!s->base) s->base = (uint8_t*)malloc(bytes);  // pageable fallback: staged by the runtime
        if (!s->base) die("error: out of host memory for read slabs");
        s->reads = s->base;
        s->pos = (int64_t*)(s->base + cap_ * read_stride());
        s->rlen = (uint16_t*)(s->base + cap_ * (read_stride() + 8));
        return s;
    }
    void put(Slab* s) {
        std::lock_guard<std::mutex> lk(m_);
        free_.push_back(s);
    }

   private:
    static void release(Slab* s) {
        if (s->pinned) msw_host_free(s->base);
        else free(s->base);
        delete s;
    }
    uint64_t cap_;
    std::mutex m_;
    std::vector<Slab*> free_;
};

struct Chunk {
    size_t file_index = 0;
    SlabPool* pool = nullptr;
    SlabPool::Slab* slab = nullptr;  // sw: reads n x read_stride(), rlen, pos
    std::vector<uint8_t> cat;        // compat: the chunk's sequences back to back (any read length)
    uint64_t n = 0;
    uint64_t first_read = 0;         // index of the chunk's first read in its file
    bool last = false;               // last chunk of its file
    const uint8_t* reads() const { return slab->reads; }
    const uint16_t* rlen() const { return slab->rlen; }
    const int64_t* pos() const { return slab->pos; }
    ~Chunk() {
        if (slab) pool->put(slab);
    }
};

struct FileState {
    std::string path;
    std::atomic<long long> score{0};
    std::atomic<unsigned long long> bases{0}, reads{0};
    std::atomic<int> outstanding{0};
    std::atomic<bool> reader_done{false}, failed{false}, finished{false};
    int scores_fd = -1;  // --scores-out: per-read records, written at the read's offset
    Clock::time_point t0;
    double ms = 0;
    std::string error;
};

class ChunkQueue {
   public:
    explicit ChunkQueue(size_t cap) : cap_(cap) {}
    void push(std::unique_ptr<Chunk> c) {
        std::unique_lock<std::mutex> lk(m_);
        cv_space_.wait(lk, [&] { return q_.size() < cap_; });
        q_.push_back(std::move(c));
        cv_item_.notify_one();
    }
    std::unique_ptr<Chunk> pop() {
        std::unique_lock<std::mutex> lk(m_);
        cv_item_.wait(lk, [&] { return !q_.empty() || closed_; });
        if (q_.empty()) return nullptr;
        auto c = std::move(q_.front());
        q_.pop_front();
        cv_space_.notify_one();
        return c;
    }
    void close() {
        std::lock_guard<std::mutex> lk(m_);
        closed_ = true;
        cv_item_.notify_all();
    }

   private:
    std::mutex m_;
    std::condition_variable cv_item_, cv_space_;
    std::deque<std::unique_ptr<Chunk>> q_;
    size_t cap_;
    bool closed_ = false;
};

// Workers set up (context, genome upload, staging buffers) before the clock
// starts: the run record's wall time covers the data, like the reference's
// per-file processing times; setup_ms reports the rest.
struct StartGate {
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    bool open = false;
    void arrive() {
        std::unique_lock<std::mutex> lk(m);
        ++arrived;
        cv.notify_all();
        cv.wait(lk, [&] { return open; });
    }
    void wait_open() {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return open; });
    }
    void release_when(int n) {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return arrived >= n; });
        open = true;
        cv.notify_all();
    }
};

struct WgsReport {
    std::vector<FileCheckpoint> results;
    double wall_ms = 0;
    unsigned long long cells = 0;
    int readers = 0;
    int host_threads = 0;
    std::vector<msw_stats_t> gpu;  // per worker: kernel time and algorithmic bytes (msw_ctx_stats)
    std::vector<int> gpu_dev;      // device ordinal of each gpu[] entry (workers may share a GPU)
    bool gpu_inflate = false;      // lane files inflated and parsed on the GPUs
    double setup_ms = 0;           // worker setup before the clock started (contexts, genome, buffers)
    double teardown_ms = 0;        // release after the last results, outside the clock
    // setup split (JSON "setup_phases", each phase's max over the workers):
    // reference_load on its own thread from the start of main, beside hip_init
    // (run_full_wgs waits for it before setup); context / genome upload /
    // result sets / lane reader
    // inside setup_ms (workers run them side by side); hip_init is filled in
    // by main (the first HIP call, before setup_ms)
    double reference_load_ms = 0, context_ms = 0, genome_ms = 0, result_sets_ms = 0, lane_reader_ms = 0;
    double kernel_load_ms = 0;  // msw_ctx_prepare: the scoring kernels' code objects, before the clock
    unsigned long long gz_in = 0, gz_out = 0;  // compressed / inflated bytes (GPU lane reader)
};

// GPU contexts of the --full-wgs workers: --num-gpus N of the visible devices,
// or the ordinals listed in MSW_DEVICES (comma separated; an ordinal may
// repeat: "0,0" runs two workers, each with its own context, on GPU 0 -- the
// multi-worker path on a one-GPU box).
std::vector<Device> worker_devices(const std::vector<Device>& devs, int n) {
    std::vector<Device> pool;
    const char* v = getenv("MSW_DEVICES");
    if (v && *v) {
        std::stringstream ss(v);
        std::string tok;
        while (std::getline(ss, tok, ',')) {
            char* end = nullptr;
            const long k = strtol(tok.c_str(), &end, 10);
            if (tok.empty() || *end || k < 0 || k >= (long)devs.size())
                die("error: MSW_DEVICES entry '" + tok + "' is not a visible GPU ordinal");
            pool.push_back(devs[(size_t)k]);
        }
    } else {
        pool = devs;
    }
    if (n < 1) die("error: --num-gpus must be >= 1");
    if (n > (int)pool.size())
        die("error: --num-gpus " + std::to_string(n) + " but only " + std::to_string(pool.size()) +
            " GPU context(s) available (visible GPUs, or MSW_DEVICES)");
    pool.resize((size_t)n);
    return pool;
}

// files: this process's lane files; gidx[i]: file i's index in the whole lane
// set (WGS_FILE_SHARD takes a subset), used for messages and the checkpoint.
// ref: the reference FASTA, already loading (sw mode; main starts it).
WgsReport run_full_wgs(const Args& a, const std::vector<Device>& devices, const std::vector<std::string>& files,
                       const std::vector<size_t>& gidx, size_t n_lane_files, Checkpoint& ckpt, ReferenceLoad& ref) {
    const uint64_t chunk = get_chunk_size_reads();
    const bool sw = a.score_mode == "sw";
    std::mutex setup_mu;
    double ph_ctx = 0, ph_gen = 0, ph_res = 0, ph_reader = 0, ph_kl = 0;  // max over workers
    auto setup_phase = [&](double c, double g, double r, double rd, double kl) {
        std::lock_guard<std::mutex> lk(setup_mu);
        ph_ctx = std::max(ph_ctx, c);
        ph_gen = std::max(ph_gen, g);
        ph_res = std::max(ph_res, r);
        ph_reader = std::max(ph_reader, rd);
        ph_kl = std::max(ph_kl, kl);
    };
    auto report_setup = [&](WgsReport& rep) {
        rep.reference_load_ms = ref.ms;
        rep.context_ms = ph_ctx;
        rep.genome_ms = ph_gen;
        rep.result_sets_ms = ph_res;
        rep.lane_reader_ms = ph_reader;
        rep.kernel_load_ms = ph_kl;
    };
    if (sw && a.reference.empty()) die("error: --score-mode sw with --full-wgs needs --reference <FASTA>");
    // the reference: loading since the top of main, beside the HIP runtime
    // init (which takes longer), so this wait is normally over at once; a
    // reference that cannot be read fails here, before any worker starts
    if (sw) printf("Loaded reference: %zu bases\n", ref.get().size());
    auto genome = [&]() -> const std::string& { return ref.get(); };
    const int ngpu = (int)devices.size();  // already worker_devices(): one worker per entry
    std::vector<msw_stats_t> gstats((size_t)ngpu);
    std::vector<std::unique_ptr<FileState>> st(files.size());
    std::vector<size_t> todo;
    for (size_t i = 0; i < files.size(); ++i) {
        st[i].reset(new FileState());
        st[i]->path = files[i];
        auto it = ckpt.files.find(gidx[i]);
        if (it != ckpt.files.end() && it->second.completed && it->second.file_path == files[i]) {
            printf("  Skipping completed file %zu/%zu: %s (score %lld)\n", gidx[i] + 1, n_lane_files,
                   files[i].c_str(), it->second.score);
        } else {
            todo.push_back(i);
        }
    }
    ChunkQueue queue(2 * (size_t)ngpu + 2);
    SlabPool slabs(chunk);
    std::mutex ck_mu;
    std::atomic<unsigned long long> cells{0};
    const auto t_setup = Clock::now();
    auto t_all = t_setup;
    StartGate gate;
    // the clock stops when the last worker has its last results on the host;
    // teardown (reader / context / genome release) is reported apart, like setup
    std::atomic<long long> t_done_ns{0};
    auto mark_done = [&]() {
        const long long t = Clock::now().time_since_epoch().count();
        long long cur = t_done_ns.load();
        while (t > cur && !t_done_ns.compare_exchange_weak(cur, t)) {
        }
    };
    // MSW_CLI_TRACE=1: per worker, ms since the start gate of each batch's
    // arrival from the reader, its submission, and its settle (stderr)
    static const bool cli_trace = getenv("MSW_CLI_TRACE") != nullptr;
    auto trace_ev = [&](int wi, const char* what, uint64_t n) {
        if (cli_trace)
            fprintf(stderr, "[cli trace] worker %d %s n=%llu t=%.3f ms\n", wi, what, (unsigned long long)n,
                    ms_since(t_all));
    };
    auto wall_and_teardown = [&](WgsReport& rep) {
        const double total = ms_since(t_all);
        const long long d = t_done_ns.load();
        rep.wall_ms = d ? std::chrono::duration<double, std::milli>(Clock::time_point(Clock::duration(d)) - t_all).count()
                        : total;
        rep.teardown_ms = total - rep.wall_ms;
    };

    auto finish_file = [&](size_t fi) {
        FileState& f = *st[fi];
        if (f.finished.exchange(true)) return;  // exactly once (reader or GPU thread)
        f.ms = ms_since(f.t0);
        if (f.scores_fd >= 0) {
            close(f.scores_fd);
            f.scores_fd = -1;
        }
        FileCheckpoint c;
        c.file_path = f.path;
        c.file_index = gidx[fi];
        c.score = f.score.load();
        c.processing_time_ms = f.ms;
        c.total_bases = f.bases.load();
        c.total_reads = f.reads.load();
        c.completed = !f.failed.load();
        std::lock_guard<std::mutex> lk(ck_mu);
        ckpt.files[gidx[fi]] = c;
        ckpt.save();
        printf("  File %zu done: %s score=%lld reads=%llu bases=%llu time=%.2fs%s\n", gidx[fi] + 1, f.path.c_str(),
               c.score, c.total_reads, c.total_bases, f.ms / 1000.0, c.completed ? "" : " (FAILED)");
        fflush(stdout);
    };

    // GPU lane reader (sw mode, every lane file BGZF, MSW_GPU_INFLATE != 0):
    // each worker takes whole files; the host reads compressed bytes only and
    // inflate, parse, window cut and scoring run on the worker's GPU
    // (msw_gfastq_* + msw_align_reads_device).  Per-read results come back to
    // the host for the i64 sums and --scores-out, one batch behind the GPU.
    bool gpu_reader = sw && env_or("MSW_GPU_INFLATE", "1") != "0" && !todo.empty();
    for (size_t fi : todo) gpu_reader = gpu_reader && msw_is_bgzf(files[fi].c_str());
    if (gpu_reader) {
        std::atomic<unsigned long long> gz_in{0}, gz_out{0};
        // reads per scoring launch; wide slabs (MSW_MAX_READ_LEN) keep a batch's
        // slab near 256 MiB (two per worker)
        // per-read records (--scores-out) are host work per read: batches of
        // 256k reads, so one batch's records are written while the next one
        // scores (config 3 from FASTQ: 17.4-18.0 -> 16.3-16.4 ms per 1 M reads,
        // profiles/r05/c3f/c3f_batch_ab.jsonl); sums only: 1 M-read batches
        const uint64_t batch_default = a.scores_out.empty() ? (1u << 20) : (1u << 18);
        const uint64_t batch = std::max<uint64_t>(
            chunk, std::min<uint64_t>(strtoull(env_or("MSW_GFASTQ_BATCH", std::to_string(batch_default)).c_str(),
                                               nullptr, 10),
                                      (256ull << 20) / read_stride()));
        std::atomic<size_t> next_file{0};
        // A claimed file is pending (prefetched by its claimer) until a worker
        // starts it; a worker left with nothing to claim takes another
        // worker's pending file instead of idling (with few or
        // uneven files the claim-ahead could leave one worker a whole file
        // of work at the end).  0 = pending, 1 = started; indexed like st.
        std::unique_ptr<std::atomic<int>[]> started(new std::atomic<int>[st.size()]);
        for (size_t i = 0; i < st.size(); ++i) started[i] = 0;
        auto start_file = [&](size_t fi) { int e = 0; return started[fi].compare_exchange_strong(e, 1); };
        std::vector<std::thread> workers;
        // two workers (contexts) per GPU by default: one file's inflate and
        // host reads overlap the other's scoring
        // (three or four workers per GPU measured slower: DESIGN.md 5)
        const int per_gpu = 2;
        const int nworkers = ngpu * per_gpu;
        gstats.assign((size_t)nworkers, msw_stats_t{});
        for (int wi = 0; wi < nworkers; ++wi) {
            workers.emplace_back([&, wi]() {
                const int gi = wi % ngpu;
                const auto ts0 = Clock::now();
                // lean: a GPU-reader worker scores device-resident batches
                // only, so its context makes just the compute stream
                Ctx ctx(devices[gi].ordinal, MSW_CTX_LEAN);
                // With per-read records (256k-read batches) the batches
                // alternate over two streams (with the two result sets), so
                // one batch's read emit and window cut run beside the other
                // batch's scoring instead of between two launches: config 3
                // from FASTQ 13.67-13.99 -> 13.25-13.74 ms.  Sums only (1 M-read
                // batches that fill the GPU alone) keep one stream: config 4
                // measured 3 % slower on two.
                void* st2 = nullptr;
                if (!a.scores_out.empty() && msw_stream_create(ctx.h, &st2) != MSW_OK)
                    die(std::string("GPU stream: ") + msw_last_error());
                void* const streams[2] = {nullptr, st2};
                const double t_ctx = ms_since(ts0);
                msw_gfastq* gr = nullptr;  // one reader per worker, reset per file (buffers kept)
                if (msw_gfastq_open(ctx.h, nullptr, read_stride(), batch, 1, 0, &gr) != MSW_OK)
                    die(std::string("GPU lane reader: ") + msw_last_error());
                const double t_rd = ms_since(ts0) - t_ctx;
                const size_t kNone = ~(size_t)0;
                size_t pending = kNone;
                auto claim = [&]() -> size_t {
                    const size_t k = next_file.fetch_add(1);
                    return k < todo.size() ? todo[k] : kNone;
                };
                // the first file: claimed now and opened / pinned on the
                // reader's thread (msw_gfastq_prefetch) while this worker
                // uploads the genome and allocates its result sets, so its
                // first window is ready when the clock starts (the same work
                // on a helper thread beside the reader's buffers measured
                // equal, and starting the prefetch later cost ~0.5 ms of the
                // timed region: profiles/r06/c3f/setup_ab.jsonl)
                pending = claim();
                if (pending != kNone) (void)msw_gfastq_prefetch(gr, st[pending]->path.c_str());
                const msw_scoring_t sc = scoring_of(a, !a.scores_out.empty());
                msw_genome* gen = nullptr;
                const auto tg0 = Clock::now();
                const std::string& ref_seq = genome();
                if (msw_genome_create(ctx.h, (const uint8_t*)ref_seq.data(), ref_seq.size(), &gen) != MSW_OK)
                    die(std::string("GPU genome upload error: ") + msw_last_error());
                const double t_gen = ms_since(tg0);
                // the scoring kernels' modules, loaded now rather than at the first batch
                const auto tk0 = Clock::now();
                if (msw_ctx_prepare(ctx.h, &sc) != MSW_OK) die(std::string("GPU kernel load: ") + msw_last_error());
                const double t_kl = ms_since(tk0);
                const auto tres0 = Clock::now();
                // two result sets: batch k's copy-back lands while batch k+1 runs
                struct Res {
                    int32_t* d_score = nullptr;
                    int16_t *d_ei = nullptr, *d_ej = nullptr;
                    uint16_t* d_wlen = nullptr;
                    uint8_t* h = nullptr;  // pinned: score i32 | ei i16 | ej i16 | rlen u16 | wlen u16
                    uint64_t n = 0, first = 0;
                    size_t fi = 0;
                    uint64_t fence = 0;  // after the batch's copy-back (msw_fence_record)
                    bool live = false;
                    uint64_t* rec = nullptr;  // --scores-out: the batch's records (recbuf)
                } res[2];
                const size_t rec = 4 + 2 + 2 + 2 + 2;
                for (Res& r : res) {
                    r.d_score = (int32_t*)msw_dev_alloc(ctx.h, batch * 4);
                    r.d_ei = (int16_t*)msw_dev_alloc(ctx.h, batch * 2);
                    r.d_ej = (int16_t*)msw_dev_alloc(ctx.h, batch * 2);
                    r.d_wlen = (uint16_t*)msw_dev_alloc(ctx.h, batch * 2);
                    r.h = (uint8_t*)msw_host_alloc(batch * rec);
                    if (!r.d_score || !r.d_ei || !r.d_ej || !r.d_wlen || !r.h)
                        die(std::string("GPU lane reader buffers: ") + msw_last_error());
                }
                // per-read records of a batch, built here and written from here:
                // allocated and touched in setup (a fresh 2 MB buffer per batch
                // page-faulted inside the last batch's settle, after the GPU)
                std::unique_ptr<uint64_t[]> recbuf;
                if (!a.scores_out.empty()) {
                    recbuf.reset(new uint64_t[2 * batch]);  // one half per result set
                    memset(recbuf.get(), 0, 2 * batch * sizeof(uint64_t));
                    res[0].rec = recbuf.get();
                    res[1].rec = recbuf.get() + batch;
                }
                const double t_res = ms_since(tres0);
                unsigned long long alg_local = 0;
                // per file this worker has open: batches in flight, reader done
                std::map<size_t, std::pair<int, bool>> open_files;
                auto maybe_finish = [&](size_t fi) {
                    auto it = open_files.find(fi);
                    if (it == open_files.end() || it->second.first > 0 || !it->second.second) return;
                    open_files.erase(it);
                    finish_file(fi);
                };
                // host side of a finished batch: sums, cells, per-read records
                // (settle_work: the batch's own buffers, the file's atomics and
                // its scores file; settle_book: this worker's file table).
                struct Settled {
                    unsigned long long alg = 0;
                };
                auto settle_work = [&](Res& r) -> Settled {
                    Settled out;
                    FileState& f = *st[r.fi];
                    trace_ev(wi, "settle-wait", r.n);
                    if (msw_fence_wait(ctx.h, r.fence) != MSW_OK) {
                        fprintf(stderr, "  GPU %d alignment error: %s\n", gi, msw_last_error());
                        f.failed = true;
                        return out;
                    }
                    const int32_t* sc32 = (const int32_t*)r.h;
                    const int16_t* ei = (const int16_t*)(r.h + batch * 4);
                    const int16_t* ej = ei + batch;
                    const uint16_t* rl = (const uint16_t*)(ej + batch);
                    const uint16_t* wl = rl + batch;
                    long long sum = 0;
                    unsigned long long cl = 0, nb = 0, nw = 0;
                    // records [score i32 | end_i i16 | end_j i16], built as whole
                    // words in the same pass as the sums
                    uint64_t* rec = f.scores_fd >= 0 ? r.rec : nullptr;
                    for (uint64_t i = 0; i < r.n; ++i) {
                        sum += sc32[i];
                        cl += (unsigned long long)rl[i] * wl[i];
                        nb += rl[i];
                        nw += wl[i];
                        if (rec)
                            rec[i] = (uint64_t)(uint32_t)sc32[i] | (uint64_t)(uint16_t)ei[i] << 32 |
                                     (uint64_t)(uint16_t)ej[i] << 48;
                    }
                    out.alg = nb + nw + (sc.want_coords ? 8ull : 4ull) * r.n;
                    f.score += sum;
                    f.bases += nb;
                    f.reads += r.n;
                    cells += cl;
                    if (rec && pwrite(f.scores_fd, rec, r.n * 8, (off_t)(r.first * 8)) != (ssize_t)(r.n * 8)) {
                        fprintf(stderr, "  error writing scores for %s\n", f.path.c_str());
                        f.failed = true;
                    }
                    return out;
                };
                auto settle_book = [&](Res& r, const Settled& o) {
                    alg_local += o.alg;
                    open_files[r.fi].first -= 1;
                    maybe_finish(r.fi);
                    trace_ev(wi, "settled", r.n);
                };
                auto settle = [&](Res& r) {
                    if (!r.live) return;
                    r.live = false;
                    settle_book(r, settle_work(r));
                };
                int cur = 0;
                setup_phase(t_ctx, t_gen, t_res, t_rd, t_kl);
                // the reader's stats of the file it just finished
                auto reader_done = [&](size_t fi) {
                    uint64_t bi = 0, bo = 0;
                    msw_gfastq_stats(gr, nullptr, nullptr, nullptr, nullptr, &bi, &bo);
                    gz_in += bi;
                    gz_out += bo;
                    st[fi]->reader_done = true;
                    open_files[fi].second = true;
                    maybe_finish(fi);
                };
                // next file for this worker: reset the reader (its compressed
                // bytes start loading in the background), false when none is
                // left.  The worker claims the file after it at the same time
                // and has the reader pin that file's first window now
                // (msw_gfastq_prefetch), so the next switch does not wait on it.
                auto open_next = [&](size_t* fi_out) -> bool {
                    for (;;) {
                        size_t fi = pending != kNone ? pending : claim();
                        pending = kNone;
                        if (fi == kNone) {  // nothing left to claim: another worker's pending file
                            for (size_t k : todo)
                                if (started[k].load() == 0 && start_file(k)) {
                                    fi = k;
                                    break;
                                }
                            if (fi == kNone) return false;
                        } else if (!start_file(fi)) {
                            continue;  // taken by an idle worker meanwhile
                        }
                        FileState& f = *st[fi];
                        f.t0 = Clock::now();
                        open_files[fi] = {0, false};
                        if (!a.scores_out.empty()) {
                            const size_t slash = f.path.find_last_of('/');
                            const std::string out = a.scores_out + "/" +
                                                    (slash == std::string::npos ? f.path : f.path.substr(slash + 1)) +
                                                    ".scores";
                            f.scores_fd = open(out.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
                            if (f.scores_fd < 0) die("error: cannot create " + out);
                        }
                        printf("  Processing file %zu/%zu: %s (GPU inflate)\n", gidx[fi] + 1, n_lane_files,
                               f.path.c_str());
                        fflush(stdout);
                        if (msw_gfastq_reset(gr, f.path.c_str()) != MSW_OK) {
                            f.error = msw_last_error();
                            fprintf(stderr, "  Error reading %s: %s\n", f.path.c_str(), f.error.c_str());
                            f.failed = true;
                            reader_done(fi);
                            continue;
                        }
                        pending = claim();
                        if (pending != kNone) (void)msw_gfastq_prefetch(gr, st[pending]->path.c_str());
                        *fi_out = fi;
                        return true;
                    }
                };
                gate.arrive();
                // One loop over the batches of all of this worker's files: a
                // file's last batches are settled after the next file's first
                // batch is launched, so the next file's read, inflate and parse
                // (reader stream) run beside this file's scoring (compute stream).
                size_t fi = 0;
                bool have = open_next(&fi);
                while (have) {
                    FileState& f = *st[fi];
                    msw_dev_reads_t d;
                    void* const bs = streams[cur];  // this batch's stream
                    if (msw_gfastq_next(gr, bs, &d) != MSW_OK) {
                        f.error = msw_last_error();
                        fprintf(stderr, "  Error reading %s: %s\n", f.path.c_str(), f.error.c_str());
                        f.failed = true;
                        reader_done(fi);
                        have = open_next(&fi);
                        continue;
                    }
                    trace_ev(wi, "batch", d.n);
                    if (d.n == 0) {
                        reader_done(fi);
                        have = open_next(&fi);
                        continue;
                    }
                    Res& r = res[cur];
                    settle(r);  // the batch before last used this result set
                    msw_out_t o{r.d_score, r.d_ei, r.d_ej};
                    if (msw_align_reads_device(ctx.h, &sc, gen, d.reads, d.read_len, d.read_stride, d.pos, d.n,
                                               a.window > 0 ? (uint32_t)a.window : 0u, d.max_len, &o, r.d_wlen,
                                               bs) != MSW_OK ||
                        msw_memcpy_d2h_async(ctx.h, r.h, r.d_score, d.n * 4, bs) != MSW_OK ||
                        // end cells only feed --scores-out records
                        (sc.want_coords &&
                         (msw_memcpy_d2h_async(ctx.h, r.h + batch * 4, r.d_ei, d.n * 2, bs) != MSW_OK ||
                          msw_memcpy_d2h_async(ctx.h, r.h + batch * 6, r.d_ej, d.n * 2, bs) != MSW_OK)) ||
                        msw_memcpy_d2h_async(ctx.h, r.h + batch * 8, d.read_len, d.n * 2, bs) != MSW_OK ||
                        msw_memcpy_d2h_async(ctx.h, r.h + batch * 10, r.d_wlen, d.n * 2, bs) != MSW_OK ||
                        msw_fence_record(ctx.h, bs, &r.fence) != MSW_OK) {
                        fprintf(stderr, "  GPU %d alignment error: %s\n", gi, msw_last_error());
                        f.failed = true;
                        (void)msw_synchronize(ctx.h);
                        reader_done(fi);
                        have = open_next(&fi);
                        continue;
                    }
                    trace_ev(wi, "submitted", d.n);
                    r.n = d.n;
                    r.first = d.first_read;
                    r.fi = fi;
                    r.live = true;
                    open_files[fi].first += 1;
                    cur ^= 1;
                }
                // (the last two batches' host work on two threads measured
                // equal: config 3 from FASTQ 13.22-13.42 vs 13.16-13.26 ms)
                settle(res[cur]);
                settle(res[cur ^ 1]);
                mark_done();
                msw_ctx_stats(ctx.h, &gstats[(size_t)wi], 0);
                gstats[(size_t)wi].alg_bytes = alg_local;
                // the reader, result sets, genome and context stay allocated:
                // the process exits (_exit in main) once the record is written
                (void)gr;
                (void)gen;
                ctx.keep = true;
            });
        }
        gate.release_when(nworkers);
        t_all = Clock::now();
        for (auto& t : workers) t.join();
        for (size_t fi : todo) finish_file(fi);
        WgsReport rep;
        rep.setup_ms = std::chrono::duration<double, std::milli>(t_all - t_setup).count();
        report_setup(rep);
        rep.gz_in = gz_in.load();
        rep.gz_out = gz_out.load();
        wall_and_teardown(rep);
        rep.cells = cells.load();
        rep.readers = 0;
        rep.host_threads = nworkers;
        rep.gpu = gstats;
        for (int wi = 0; wi < nworkers; ++wi) rep.gpu_dev.push_back(devices[wi % ngpu].ordinal);
        rep.gpu_inflate = true;
        for (size_t i = 0; i < files.size(); ++i)
            if (ckpt.files.count(gidx[i])) rep.results.push_back(ckpt.files[gidx[i]]);
        return rep;
    }

    // Readers: one thread per lane file in flight (a gzip stream inflates on
    // one core; zlib gives ~0.5-0.75 M reads/s per thread, far below what one
    // GPU scores, so the host side wants every file open at once):
    // min(files, MSW_HOST_THREADS), by default the CPUs this process may use
    // (usable_cpus()).
    std::atomic<size_t> next_file{0};
    const int host_threads =
        std::max(1, atoi(env_or("MSW_HOST_THREADS", std::to_string(usable_cpus())).c_str()));
    const int nreaders = std::max(1, std::min<int>((int)todo.size(), std::max(host_threads, 2 * ngpu)));
    // Fewer files than the CPU share: BGZF blocks of one file inflate on
    // several threads (msw_fastq.cpp; MSW_INFLATE_THREADS overrides).
    if (!getenv("MSW_INFLATE_THREADS")) {
        const std::string per = std::to_string(std::max(1, host_threads / nreaders));
        setenv("MSW_INFLATE_THREADS", per.c_str(), 0);
    }
    std::vector<std::thread> readers;
    std::atomic<int> readers_left{nreaders};
    for (int r = 0; r < nreaders; ++r) {
        readers.emplace_back([&]() {
            gate.wait_open();
            for (;;) {
                const size_t k = next_file.fetch_add(1);
                if (k >= todo.size()) break;
                const size_t fi = todo[k];
                FileState& f = *st[fi];
                f.t0 = Clock::now();
                if (sw && !a.scores_out.empty()) {
                    const size_t slash = f.path.find_last_of('/');
                    const std::string out = a.scores_out + "/" +
                                            (slash == std::string::npos ? f.path : f.path.substr(slash + 1)) + ".scores";
                    f.scores_fd = open(out.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
                    if (f.scores_fd < 0) die("error: cannot create " + out);
                }
                printf("  Processing file %zu/%zu: %s\n", gidx[fi] + 1, n_lane_files, f.path.c_str());
                fflush(stdout);
                msw_fastq* fq = nullptr;
                if (msw_fastq_open(f.path.c_str(), &fq) != MSW_OK) {
                    f.error = msw_last_error();
                    f.failed = true;
                    f.reader_done = true;
                    if (f.outstanding.load() == 0) finish_file(fi);
                    continue;
                }
                uint64_t reads_so_far = 0;
                for (;;) {
                    std::unique_ptr<Chunk> c(new Chunk());
                    c->file_index = fi;
                    c->first_read = reads_so_far;
                    bool ok = true;
                    if (sw) {
                        c->pool = &slabs;
                        c->slab = slabs.get();
                        ok = msw_fastq_next(fq, c->slab->reads, c->slab->rlen, read_stride(), chunk, &c->n,
                                            c->slab->pos) == MSW_OK;
                    } else {
                        // compat: exactly `chunk` reads of any length, concatenated
                        // (aligner.rs:270); the buffer grows when a read does not fit
                        std::vector<uint8_t>& cat = c->cat;
                        cat.resize((size_t)std::min<uint64_t>(chunk, 65536) * 160);
                        std::vector<uint32_t> lens((size_t)std::min<uint64_t>(chunk, 65536));
                        uint64_t used = 0;
                        while (ok && c->n < chunk) {
                            uint64_t got = 0, nb = 0, need = 0;
                            const uint64_t want = std::min<uint64_t>(chunk - c->n, lens.size());
                            ok = msw_fastq_next_packed(fq, cat.data() + used, cat.size() - used, lens.data(), want,
                                                       &got, &nb, &need) == MSW_OK;
                            used += nb;
                            c->n += got;
                            if (ok && need) cat.resize(std::max(2 * cat.size(), (size_t)(used + need)));
                            else if (ok && got < want) break;  // end of file
                        }
                        cat.resize((size_t)used);
                    }
                    if (!ok) {
                        f.error = msw_last_error();
                        fprintf(stderr, "  Error reading %s: %s\n", f.path.c_str(), f.error.c_str());
                        f.failed = true;
                        break;
                    }
                    if (c->n == 0) break;
                    reads_so_far += c->n;
                    f.outstanding.fetch_add(1);
                    queue.push(std::move(c));
                }
                msw_fastq_close(fq);
                f.reader_done = true;
                // A file with no chunks in flight is finished here; otherwise by the GPU thread.
                if (f.outstanding.load() == 0) finish_file(fi);
            }
            if (readers_left.fetch_sub(1) == 1) queue.close();
        });
    }

    std::vector<std::thread> workers;
    for (int g = 0; g < ngpu; ++g) {
        workers.emplace_back([&, g]() {
            const auto ts0 = Clock::now();
            Ctx ctx(devices[g].ordinal);
            const double t_ctx = ms_since(ts0);
            const msw_scoring_t sc = scoring_of(a, !a.scores_out.empty());
            // sw mode: the reference genome lives in this GPU's HBM; a chunk
            // ships reads + window positions, windows are cut on the GPU.
            msw_genome* gen = nullptr;
            const uint64_t gsize = sw ? genome().size() : 0;
            if (sw && msw_genome_create(ctx.h, (const uint8_t*)genome().data(), gsize, &gen) != MSW_OK)
                die(std::string("GPU genome upload error: ") + msw_last_error());
            const double t_gen = ms_since(ts0);
            if (msw_ctx_prepare(ctx.h, &sc) != MSW_OK) die(std::string("GPU kernel load: ") + msw_last_error());
            setup_phase(t_ctx, t_gen - t_ctx, 0.0, 0.0, ms_since(ts0) - t_gen);
            gate.arrive();
            // Up to three chunks in flight (msw_align_reads_async; msw_wait on the
            // oldest ticket before a fourth is staged): the context's three
            // staging slots keep uploads of chunk k+1 under kernel k.
            struct InFlight {
                std::unique_ptr<Chunk> c;
                std::vector<uint16_t> want;
                std::vector<int32_t> score;
                std::vector<int16_t> ei, ej;
                uint64_t ticket = 0;
                unsigned long long cells = 0, bases = 0;
                bool failed = false;
            };
            auto settle = [&](InFlight& fl) {
                FileState& f = *st[fl.c->file_index];
                long long chunk_score = 0;
                if (!fl.failed && fl.ticket && msw_wait(ctx.h, fl.ticket) != MSW_OK) {
                    fprintf(stderr, "  GPU %d alignment error: %s\n", g, msw_last_error());
                    fl.failed = true;
                }
                if (fl.failed) {
                    f.failed = true;
                } else {
                    for (uint64_t i = 0; i < fl.c->n; ++i) chunk_score += fl.score[i];
                    cells += fl.cells;
                    if (f.scores_fd >= 0) {
                        // chunks of one file may finish on different GPUs in any
                        // order: each lands at its reads' own offset
                        std::vector<uint8_t> rec(fl.c->n * 8);
                        for (uint64_t i = 0; i < fl.c->n; ++i) {
                            memcpy(&rec[i * 8], &fl.score[i], 4);
                            memcpy(&rec[i * 8 + 4], &fl.ei[i], 2);
                            memcpy(&rec[i * 8 + 6], &fl.ej[i], 2);
                        }
                        if (pwrite(f.scores_fd, rec.data(), rec.size(), (off_t)(fl.c->first_read * 8)) !=
                            (ssize_t)rec.size()) {
                            fprintf(stderr, "  error writing scores for %s\n", f.path.c_str());
                            f.failed = true;
                        }
                    }
                }
                f.score += chunk_score;
                f.bases += fl.bases;
                f.reads += fl.c->n;
                if (f.outstanding.fetch_sub(1) == 1 && f.reader_done.load()) finish_file(fl.c->file_index);
                fl.c.reset();
            };
            std::deque<std::unique_ptr<InFlight>> pending;
            constexpr size_t kDepth = 3;
            for (;;) {
                std::unique_ptr<Chunk> c = queue.pop();
                if (!c) break;
                FileState& f = *st[c->file_index];
                unsigned long long nb = 0;
                if (sw)
                    for (uint64_t i = 0; i < c->n; ++i) nb += c->rlen()[i];
                else
                    nb = c->cat.size();
                if (sw) {
                    // window = reference[pos : pos + W] (W = --window, at most
                    // 32767, or 2 x read length capped at 4096), clipped at the genome end
                    std::unique_ptr<InFlight> fl(new InFlight());
                    fl->bases = nb;
                    fl->want.resize(c->n);
                    fl->score.assign(c->n, 0);
                    fl->ei.assign(c->n, 0);
                    fl->ej.assign(c->n, 0);
                    for (uint64_t i = 0; i < c->n; ++i) {
                        const uint32_t w = a.window > 0 ? std::min<uint32_t>((uint32_t)a.window, 32767u)
                                                        : std::min<uint32_t>(2u * c->rlen()[i], 4096u);
                        fl->want[i] = (uint16_t)w;
                        const int64_t p = c->pos()[i];
                        if (p >= 0 && (uint64_t)p < gsize)
                            fl->cells += (unsigned long long)std::min<uint64_t>(w, gsize - (uint64_t)p) * c->rlen()[i];
                    }
                    msw_read_batch_t rb{c->reads(), c->rlen(), read_stride(), c->pos(), fl->want.data(), c->n};
                    msw_out_t o{fl->score.data(), fl->ei.data(), fl->ej.data()};
                    fl->c = std::move(c);
                    if (msw_align_reads_async(ctx.h, &sc, gen, &rb, &o, 0, &fl->ticket) != MSW_OK) {
                        fprintf(stderr, "  GPU %d alignment error: %s\n", g, msw_last_error());
                        fl->failed = true;
                    }
                    pending.push_back(std::move(fl));
                    if (pending.size() >= kDepth) {
                        settle(*pending.front());
                        pending.pop_front();
                    }
                } else {
                    // compat: chunk concat self-aligned (aligner.rs:269-276, :365-373)
                    long long chunk_score = 0;
                    const std::vector<uint8_t>& cat = c->cat;
                    if (cat.size() >= 1000) {
                        int32_t s = 0;
                        if (msw_align_compat(ctx.h, cat.data(), cat.size(), cat.data(),
                                             cat.size(), std::min<uint32_t>(devices[g].max_wg, 1024), 1000000,
                                             &s) != MSW_OK) {
                            fprintf(stderr, "  GPU %d alignment error: %s\n", g, msw_last_error());
                            f.failed = true;
                        }
                        chunk_score = s;
                    }
                    f.score += chunk_score;
                    f.bases += nb;
                    f.reads += c->n;
                    if (f.outstanding.fetch_sub(1) == 1 && f.reader_done.load()) finish_file(c->file_index);
                }
            }
            while (!pending.empty()) {
                settle(*pending.front());
                pending.pop_front();
            }
            mark_done();
            msw_ctx_stats(ctx.h, &gstats[(size_t)g], 0);
            (void)gen;  // left to the process exit, like the context (Ctx::keep)
            ctx.keep = true;
        });
    }
    gate.release_when(ngpu);
    t_all = Clock::now();
    for (auto& t : readers) t.join();
    for (auto& t : workers) t.join();
    for (size_t fi : todo) finish_file(fi);  // no-op for files already finished
    WgsReport rep;
    rep.setup_ms = std::chrono::duration<double, std::milli>(t_all - t_setup).count();
    report_setup(rep);
    wall_and_teardown(rep);
    rep.cells = cells.load();
    rep.readers = nreaders;
    rep.host_threads = host_threads;
    rep.gpu = gstats;
    for (const Device& d : devices) rep.gpu_dev.push_back(d.ordinal);
    for (size_t i = 0; i < files.size(); ++i)
        if (ckpt.files.count(gidx[i])) rep.results.push_back(ckpt.files[gidx[i]]);
    return rep;
}

std::string stable_run_id(const std::string& dir, const std::string& sample, const Args& a) {
    const char* v = getenv("WGS_RUN_ID");
    if (v && *v) return v;
    // FNV-1a over the inputs that define the run: same dataset + mode -> same id.
    // The scoring scheme and window are part of it: a checkpoint written under
    // other parameters is never resumed into this run.
    std::string key = dir + "|" + sample + "|" + a.score_mode + "|" + a.gap_model + "|" + a.reference + "|" +
                      env_or("GPU_CHUNK_SIZE_READS", "") + "|" + std::to_string(a.match) + "|" +
                      std::to_string(a.mismatch) + "|" + std::to_string(a.gap_open) + "|" +
                      std::to_string(a.gap_extend) + "|" + std::to_string(a.window) + "|" +
                      env_or("WGS_FILE_SHARD", "");
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : key) { h ^= c; h *= 1099511628211ull; }
    char buf[32];
    snprintf(buf, sizeof(buf), "wgs_%016llx", (unsigned long long)h);
    return buf;
}

void write_json(const std::string& path, const std::string& body) {
    if (path.empty()) return;
    std::ofstream f(path);
    f << body;
}

}  // namespace

// CLOCK_REALTIME in ns: the run record's process timeline (t_main_unix_ns,
// t_record_unix_ns), so a parent can split its child's wall into start-up
// (exec -> main), main -> record and exit (record -> reaped).
long long unix_ns() {
    timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    return (long long)t.tv_sec * 1000000000ll + t.tv_nsec;
}

int main(int argc, char** argv) {
    const long long t_main_ns = unix_ns();
    load_dotenv();
    const Args a = parse_args(argc, argv);
    // --full-wgs sw: the reference loads beside the HIP runtime init
    // (setup_phases.reference_load_ms is its own duration)
    ReferenceLoad ref;
    if (a.full_wgs && a.score_mode == "sw" && !a.reference.empty()) ref.start(a.reference);
    const auto t_hip = Clock::now();
    const auto devices = get_gpu_devices();  // the first HIP call: runtime init
    const double hip_init_ms = ms_since(t_hip);
    printf("Detecting system information...\n");
    for (const auto& d : devices) printf("  GPU %d: %s (%.1f GB)\n", d.ordinal, d.name.c_str(), d.memory_gb);
    if (devices.empty()) printf("  No GPU detected\n");

    if (a.full_wgs) {
        printf("Processing FULL WGS dataset...\n");
        if (!a.gpu || !is_gpu_available()) die("error: gpu acceleration is required for full WGS processing");
        const std::string dir = env_or("WGS_DATA_DIR", "/path/to/wgs/data");
        const std::string sample = env_or("WGS_SAMPLE_ID", "SAMPLE_ID");
        const int lanes = atoi(env_or("WGS_LANES", "8").c_str()) > 0 ? atoi(env_or("WGS_LANES", "8").c_str()) : 8;
        const int rpl = atoi(env_or("WGS_READS_PER_LANE", "2").c_str()) > 0
                            ? atoi(env_or("WGS_READS_PER_LANE", "2").c_str()) : 2;
        std::vector<std::string> files;
        for (int lane = 1; lane <= lanes; ++lane)
            for (int r = 1; r <= rpl; ++r) {
                char name[512];
                snprintf(name, sizeof(name), "%s/%s_L%03d_R%d_001.fastq.gz", dir.c_str(), sample.c_str(), lane, r);
                files.push_back(name);
            }
        const size_t n_lane_files = files.size();
        std::vector<size_t> gidx(files.size());
        for (size_t i = 0; i < gidx.size(); ++i) gidx[i] = i;
        // WGS_FILE_SHARD=r/N: this process takes lane files r, r+N, r+2N, ...
        // (one process per GPU, e.g. bench.py's config-4 leg under
        // torch.distributed.run; the reference has no multi-GPU path, gpu.rs:117,125)
        const std::string shard = env_or("WGS_FILE_SHARD", "");
        if (!shard.empty()) {
            int r = -1, n = 0;
            char tail = 0;
            if (sscanf(shard.c_str(), "%d/%d%c", &r, &n, &tail) != 2 || n < 1 || r < 0 || r >= n)
                die("error: WGS_FILE_SHARD must be r/N with 0 <= r < N, got '" + shard + "'");
            std::vector<std::string> mine;
            std::vector<size_t> mine_idx;
            for (size_t i = (size_t)r; i < files.size(); i += (size_t)n) {
                mine.push_back(files[i]);
                mine_idx.push_back(i);
            }
            files.swap(mine);
            gidx.swap(mine_idx);
            printf("File shard %d/%d: %zu lane file(s)\n", r, n, files.size());
        }
        Checkpoint ck;
        ck.run_id = stable_run_id(dir, sample, a);
        ck.path = a.checkpoint_dir + "/checkpoint_" + ck.run_id + ".json";
        ck.total_files = files.size();
        if (ck.load()) printf("Resuming run %s from %s\n", ck.run_id.c_str(), ck.path.c_str());
        const std::vector<Device> workers = worker_devices(devices, a.num_gpus);
        const WgsReport rep = run_full_wgs(a, workers, files, gidx, n_lane_files, ck, ref);
        long long total = 0;
        unsigned long long reads = 0, bases = 0;
        bool all_ok = true;
        printf("\nFULL WGS PROCESSING COMPLETE\n==========================================\n");
        printf("Total files processed: %zu\n", rep.results.size());
        for (const auto& r : rep.results) {
            printf("File %zu: Score=%lld, Time=%.2fs\n", r.file_index + 1, r.score, r.processing_time_ms / 1000.0);
            total += r.score;
            reads += r.total_reads;
            bases += r.total_bases;
            all_ok = all_ok && r.completed;
        }
        printf("Total reads: %llu, total bases: %llu, total score: %lld\n", reads, bases, total);
        printf("Wall time: %.2f s", rep.wall_ms / 1000.0);
        if (rep.cells) printf(", %.1f GCUPS end-to-end", rep.cells / (rep.wall_ms * 1e6));
        printf("\n");
        // Run record: the reference's BenchmarkResult fields (tools/benchmark.rs:17-34;
        // its fake gpu_utilization_avg / gpu_memory_used_mb are dropped) plus GCUPS
        // (kernel and end to end), HBM GB/s and roofline fractions.
        const double secs = std::max(rep.wall_ms / 1000.0, 1e-9);
        char ts[64];
        {
            const time_t now = time(nullptr);
            struct tm tmv;
            gmtime_r(&now, &tmv);
            strftime(ts, sizeof(ts), "%Y-%m-%dT%H:%M:%SZ", &tmv);
        }
        double ram_gb = 0;
        {
            std::ifstream mi("/proc/meminfo");
            std::string k;
            double v = 0;
            if (mi >> k >> v && k == "MemTotal:") ram_gb = v / (1024.0 * 1024.0);
        }
        const double gcups_e2e = rep.cells ? rep.cells / (rep.wall_ms * 1e6) : 0.0;
        // Kernel rate: the job's cells over the busiest GPU's kernel time
        // (HIP events around every chunk's scoring launch, msw_ctx_stats),
        // the kernel time of the workers sharing a GPU summed.
        double kmax = 0, ksum = 0;
        unsigned long long alg = 0;
        std::map<int, double> per_dev;
        for (size_t i = 0; i < rep.gpu.size(); ++i) {
            per_dev[i < rep.gpu_dev.size() ? rep.gpu_dev[i] : (int)i] += rep.gpu[i].kernel_ms;
            ksum += rep.gpu[i].kernel_ms;
            alg += rep.gpu[i].alg_bytes;
        }
        for (const auto& kv : per_dev) kmax = std::max(kmax, kv.second);
        const int ng = (int)per_dev.size();  // physical GPUs
        const bool sw_mode = a.score_mode == "sw";
        const double gcups = kmax > 0 && sw_mode ? rep.cells / (kmax * 1e6) : 0.0;
        const double hbm_gbps = kmax > 0 ? alg / (kmax * 1e6) : 0.0;
        // Per-GPU ceilings: 8 TB/s HBM; VALU issue of the loop that ran (128
        // cells per 19.16 / 30.28 / 35.88 / 46.99 cycles per packed row-step for
        // linear / +coords / affine / +coords, x 1024 SIMDs x 2.4 GHz; bench.py
        // CYCLES_PER_ROW_STEP).
        const bool coords = !a.scores_out.empty();
        const double valu_ceiling = a.gap_model == "affine" ? (coords ? 6694.5 : 8767.6)
                                                            : (coords ? 10389.5 : 16418.2);
        const double frac_hbm = ng ? hbm_gbps / (8000.0 * ng) : 0.0;
        const double frac_valu = ng && sw_mode ? gcups / (valu_ceiling * ng) : 0.0;
        // Scoring time per GPU over the wall: each worker's kernel_ms is the
        // union of its own launches, but two workers on one GPU overlap, so
        // their sum can exceed the wall -- capped at 1 (an upper bound then).
        const double busy = ng && rep.wall_ms > 0 ? std::min(1.0, ksum / (ng * rep.wall_ms)) : 0.0;
        std::ostringstream j;
        j << "{\"timestamp\": \"" << ts << "\", \"run_id\": \"" << ck.run_id << "\", \"mode\": \"full_wgs\""
          << ", \"score_mode\": \"" << a.score_mode << "\", \"files_processed\": " << rep.results.size()
          << ", \"total_files\": " << files.size() << ", \"total_reads\": " << reads << ", \"total_bases\": " << bases
          << ", \"total_score\": " << total << ", \"total_time_seconds\": " << secs << ", \"wall_ms\": " << rep.wall_ms
          << ", \"throughput_reads_per_second\": " << reads / secs
          << ", \"throughput_bases_per_second\": " << bases / secs << ", \"chunk_size\": " << get_chunk_size_reads()
          << ", \"cpu_cores_used\": " << usable_cpus() << ", \"host_reader_threads\": " << rep.readers
          << ", \"parallel_files\": " << (rep.readers > 1 || rep.host_threads > 1 ? "true" : "false")
          << ", \"system_info\": {\"gpu_name\": \"" << json_escape(devices.empty() ? "" : devices[0].name)
          << "\", \"gpu_memory_gb\": " << (devices.empty() ? 0.0 : devices[0].memory_gb)
          << ", \"cpu_cores\": " << std::thread::hardware_concurrency() << ", \"total_ram_gb\": " << ram_gb << "}"
          << ", \"num_gpus\": " << workers.size() << ", \"physical_gpus\": " << ng << ", \"host_cores\": " << std::thread::hardware_concurrency()
          << ", \"host_cpus_usable\": " << usable_cpus() << ", \"host_threads\": " << rep.host_threads
          << ", \"cells\": " << rep.cells << ", \"gcups\": " << gcups << ", \"gcups_end_to_end\": " << gcups_e2e
          << ", \"kernel_ms\": " << kmax << ", \"gpu_busy_fraction\": " << busy
          << ", \"alg_bytes\": " << alg << ", \"hbm_gbps\": " << hbm_gbps
          << ", \"roofline_fraction_hbm\": " << frac_hbm << ", \"roofline_fraction_valu\": " << frac_valu
          << ", \"gpu_inflate\": " << (rep.gpu_inflate ? "true" : "false") << ", \"setup_ms\": " << rep.setup_ms
          << ", \"setup_phases\": {\"hip_init_ms\": " << hip_init_ms << ", \"reference_load_ms\": " << rep.reference_load_ms
          << ", \"context_ms\": " << rep.context_ms << ", \"genome_ms\": " << rep.genome_ms
          << ", \"result_sets_ms\": " << rep.result_sets_ms << ", \"lane_reader_ms\": " << rep.lane_reader_ms
          << ", \"kernel_load_ms\": " << rep.kernel_load_ms << "}"
          << ", \"teardown_ms\": " << rep.teardown_ms
          << ", \"inflate_bytes_in\": " << rep.gz_in << ", \"inflate_bytes_out\": " << rep.gz_out
          << ", \"reads_per_second\": " << reads / secs << ", \"t_main_unix_ns\": " << t_main_ns
          << ", \"t_record_unix_ns\": " << unix_ns() << "}\n";
        write_json(a.json, j.str());
        // Records, scores files and checkpoint are written and closed: end the
        // process here.  The workers' contexts, genomes and pinned buffers are
        // released by the exit itself (Ctx::keep), not call by call.
        // Under rocprofv3 (its tool library is named in the environment) the
        // ordinary exit runs, so the profiler's exit handlers write its
        // output; the contexts are still left to the runtime's own exit.
        fflush(stdout);
        fflush(stderr);
        if (getenv("ROCP_TOOL_LIBRARIES") || getenv("ROCPROF_OUTPUT_PATH")) exit(all_ok ? 0 : 1);
        _exit(all_ok ? 0 : 1);
    }

    if (a.test_wgs) {
        printf("Testing WGS file reading from configured directory...\n");
        const std::string dir = env_or("WGS_DATA_DIR", "/path/to/wgs/data");
        const std::string sample = env_or("WGS_SAMPLE_ID", "SAMPLE_ID");
        for (const char* rr : {"R1", "R2"}) {
            const std::string file = sample + "_L001_" + rr + "_001.fastq.gz";
            const std::string full = dir + "/" + file;
            printf("Testing: %s\n", full.c_str());
            uint64_t bases = 0, reads = 0;
            get_chunk_size_reads();  // count_bases_in_fastq needs it (aligner.rs:538)
            if (msw_fastq_count_bases(full.c_str(), &bases, &reads) == MSW_OK)
                printf("✅ Successfully counted %llu bases in %s\n", (unsigned long long)bases, file.c_str());
            else
                printf("❌ Error counting bases in %s: %s\n", file.c_str(), msw_last_error());
        }
        return 0;
    }

    if (!a.has_seq1) die("--seq1 is required when not in test mode");
    if (!a.has_seq2) die("--seq2 is required when not in test mode");
    if (!a.gpu || !is_gpu_available()) die("error: gpu acceleration is required and no compatible gpu was found");
    printf("GPU acceleration enabled\n");
    for (const auto& d : devices) printf("  Found GPU: %s (%g GB)\n", d.name.c_str(), d.memory_gb);
    const Device& dev = devices[0];
    Ctx ctx(dev.ordinal);

    if (a.files) {
        // gpu_align_pair (aligner.rs:376-407)
        uint64_t b1 = 0, b2 = 0, r = 0;
        const uint64_t chunk = get_chunk_size_reads();
        if (msw_fastq_count_bases(a.seq1.c_str(), &b1, &r) || msw_fastq_count_bases(a.seq2.c_str(), &b2, &r)) {
            fprintf(stderr, "GPU alignment error: %s\n", msw_last_error());
            return 1;
        }
        printf("Loaded %llu bases from %s\n", (unsigned long long)b1, a.seq1.c_str());
        printf("Loaded %llu bases from %s\n", (unsigned long long)b2, a.seq2.c_str());
        const auto t0 = Clock::now();
        // File 2's chunks are cached (the reference re-decompresses file 2 once
        // per chunk of file 1, aligner.rs:390-398; the sum is identical).
        std::vector<std::string> chunks2;
        for_each_fastq_chunk(a.seq2, chunk, [&](std::string& c) { chunks2.push_back(c); return 0; });
        int32_t total = 0;  // i32 sum, wrapping like a release build
        std::string err;
        const int rc = for_each_fastq_chunk(a.seq1, chunk, [&](std::string& c1) {
            for (const auto& c2 : chunks2) {
                bool ok = false;
                const int32_t s = gpu_align(ctx, c1, c2, dev, &ok, &err);
                if (!ok) return 1;
                total = (int32_t)((uint32_t)total + (uint32_t)s);
            }
            return 0;
        });
        if (rc) {
            fprintf(stderr, "GPU alignment error: %s\n", err.empty() ? msw_last_error() : err.c_str());
            return 1;
        }
        printf("GPU Alignment Result:\n  Score: %d\n  Processing time: %.2f ms\n  GPU device: %s\n", total,
               (double)(long long)ms_since(t0), dev.name.c_str());
        return 0;
    }

    if (a.score_mode == "sw") {
        msw_scoring_t sc = scoring_of(a, true);
        const size_t rs = std::max<size_t>(16, (a.seq1.size() + 15) / 16 * 16);
        const size_t ws = std::max<size_t>(16, (a.seq2.size() + 15) / 16 * 16);
        std::vector<uint8_t> r(rs, 0), w(ws, 0);
        memcpy(r.data(), a.seq1.data(), a.seq1.size());
        memcpy(w.data(), a.seq2.data(), a.seq2.size());
        if (a.seq1.size() > 32767 || a.seq2.size() > 32767) {
            fprintf(stderr, "GPU alignment error: sequence of %zu / %zu bases exceeds the kernel limits "
                            "(read <= 32767, window <= 32767)\n", a.seq1.size(), a.seq2.size());
            return 1;
        }
        uint16_t rl = (uint16_t)a.seq1.size(), wl = (uint16_t)a.seq2.size();
        int32_t score = 0;
        int16_t ei = -1, ej = -1;
        msw_batch_t b{r.data(), w.data(), &rl, &wl, (uint32_t)rs, (uint32_t)ws, 1};
        msw_out_t o{&score, &ei, &ej};
        if (msw_align_batch(ctx.h, &sc, &b, &o, 0) != MSW_OK) {
            fprintf(stderr, "GPU alignment error: %s\n", msw_last_error());
            return 1;
        }
        printf("GPU Alignment score: %d\n", score);
        printf("Best cell: read %d, window %d\n", ei, ej);
        return 0;
    }
    bool ok = false;
    std::string err;
    const int32_t score = gpu_align(ctx, a.seq1, a.seq2, dev, &ok, &err);
    if (!ok) {
        fprintf(stderr, "GPU alignment error: %s\n", err.c_str());
        return 1;
    }
    printf("GPU Alignment score: %d\n", score);
    return 0;
}
