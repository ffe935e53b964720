// weighted_ld — the reference CLI (rust/weighted_ld/src/main.rs) rebuilt on the
// C ABI of libweightedld.so.  Same flags (main.rs:14-68), same pipeline
// (main.rs:121-213), same TSV files (main.rs:70-119) and the same env_logger
// style log lines on stderr; the all-pairs step runs on the GPU.
//
// Additions (do not change the reference flags' meaning):
//   --vcf-input PATH   VCF input following WeightedLD.py's handle_vcf (no site
//                      filter, site index = POS), for BASELINE config 3
//   --device N         HIP device ordinal (default 0)
//   --devices G|LIST   shard the pair space over G devices (0..G-1) or a comma
//                      list of ordinals (repeats allowed) in this one process
//                      (wld_create_multi); overrides --device
//   --kernel K         auto | valu | mfma (default auto)
#include <chrono>
#include <cinttypes>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <thread>

#include <sys/ioctl.h>
#include <unistd.h>
#include <vector>

#include "weightedld.h"
#include "tsv_format.hpp"

namespace {

int g_level = 3;  // 0 off, 1 error, 2 warn, 3 info, 4 debug, 5 trace

void init_logger() {
    const char *e = getenv("RUST_LOG");  // env_logger, default_filter_or("info") (main.rs:122)
    if (!e || !*e) return;
    std::string s(e);
    for (auto &c : s) c = (char)tolower(c);
    if (s.find("trace") != std::string::npos) g_level = 5;
    else if (s.find("debug") != std::string::npos) g_level = 4;
    else if (s.find("info") != std::string::npos) g_level = 3;
    else if (s.find("warn") != std::string::npos) g_level = 2;
    else if (s.find("error") != std::string::npos) g_level = 1;
    else if (s.find("off") != std::string::npos) g_level = 0;
}

void log_at(int level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void log_at(int level, const char *fmt, ...) {
    if (level > g_level) return;
    static const char *names[] = {"", "ERROR", "WARN ", "INFO ", "DEBUG", "TRACE"};
    char ts[32];
    time_t t = time(nullptr);
    struct tm g;
    gmtime_r(&t, &g);
    strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%SZ", &g);
    char msg[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    fprintf(stderr, "[%s %s weighted_ld] %s\n", ts, names[level], msg);
}
#define INFO(...) log_at(3, __VA_ARGS__)

// Rust's Debug for std::time::Duration
std::string fmt_duration(std::chrono::nanoseconds d) {
    uint64_t ns = (uint64_t)d.count();
    auto frac = [](uint64_t whole, uint64_t rem, int digits, const char *unit) {
        char buf[64];
        if (rem == 0) {
            snprintf(buf, sizeof buf, "%" PRIu64 "%s", whole, unit);
        } else {
            char f[16];
            snprintf(f, sizeof f, "%0*" PRIu64, digits, rem);
            int n = (int)strlen(f);
            while (n > 0 && f[n - 1] == '0') f[--n] = 0;
            snprintf(buf, sizeof buf, "%" PRIu64 ".%s%s", whole, f, unit);
        }
        return std::string(buf);
    };
    if (ns >= 1000000000ull) return frac(ns / 1000000000ull, ns % 1000000000ull, 9, "s");
    if (ns >= 1000000ull) return frac(ns / 1000000ull, ns % 1000000ull, 6, "ms");
    if (ns >= 1000ull) return frac(ns / 1000ull, ns % 1000ull, 3, "\xC2\xB5s");
    return frac(ns, 0, 0, "ns");
}

// human_format::Formatter::new() (2 decimals, SI prefixes)
std::string human(double v, const char *units = "") {
    static const char *pre[] = {"", "K", "M", "G", "T", "P", "E", "Z", "Y"};
    int k = 0;
    double x = v;
    while (std::fabs(x) >= 1000.0 && k < 8) {
        x /= 1000.0;
        ++k;
    }
    char buf[64];
    snprintf(buf, sizeof buf, "%.2f %s%s", x, pre[k], units);
    return buf;
}

// indicatif 0.15's ProgressBar as main.rs sets it up (main.rs:89-97, 170-178):
// template "{spinner:.green} [{elapsed_precise}] [{wide_bar:.cyan/blue}]
// {percent}% ({per_sec} {eta_precise})", progress chars "#>-", drawn on stderr
// only when the log level enables info (log_enabled!(Level::Info)) and stderr
// is a terminal (indicatif's stderr target draws nothing otherwise), at most
// 15 frames a second; dropped unfinished, it clears its line.  So TSVs and
// log lines are byte-identical whether or not a bar was drawn.
// (WLD_FORCE_PROGRESS_BAR=1 draws on a non-terminal stderr too: the tests'
// hook, where no pseudo-terminal is available.)
class ProgressBar {
  public:
    explicit ProgressBar(uint64_t len)
        : len_(len), on_(g_level >= 3 && (isatty(2) || forced())), start_(std::chrono::steady_clock::now()),
          last_(start_) {}
    ~ProgressBar() {
        if (on_ && drawn_) fputs("\r\x1b[2K", stderr), fflush(stderr);
    }
    void set_position(uint64_t pos) {
        ++updates_;
        last_pos_ = pos;
        pos_ = std::min(pos, len_);
        if (!on_) return;
        const auto now = std::chrono::steady_clock::now();
        if (drawn_ && now - last_ < std::chrono::milliseconds(66)) return;  // indicatif's 15 Hz draw rate
        last_ = now;
        draw(now);
    }
    uint64_t updates() const { return updates_; }
    uint64_t last_position() const { return last_pos_; }

  private:
    static bool forced() {
        const char *e = getenv("WLD_FORCE_PROGRESS_BAR");
        return e && *e == '1';
    }
    static std::string hms(uint64_t secs) {
        char b[32];
        snprintf(b, sizeof b, "%02" PRIu64 ":%02" PRIu64 ":%02" PRIu64, secs / 3600, secs / 60 % 60, secs % 60);
        return b;
    }
    void draw(std::chrono::steady_clock::time_point now) {
        static const char *ticks[] = {"\u2801", "\u2802", "\u2804", "\u2840", "\u2880",
                                      "\u2820", "\u2810", "\u2808"};  // indicatif's default tick chars
        const double el = std::chrono::duration<double>(now - start_).count();
        const double frac = len_ ? (double)pos_ / (double)len_ : 1.0;
        const uint64_t per_sec = el > 0.0 ? (uint64_t)((double)pos_ / el) : 0;
        const uint64_t eta = pos_ && per_sec ? (uint64_t)((double)(len_ - pos_) / (double)per_sec) : 0;
        char tail[96];
        snprintf(tail, sizeof tail, "] %d%% (%" PRIu64 "/s %s)", (int)(frac * 100.0), per_sec, hms(eta).c_str());
        struct winsize ws{};
        const int cols = ioctl(2, TIOCGWINSZ, &ws) == 0 && ws.ws_col ? ws.ws_col : 80;
        const int width = std::max(1, cols - 14 - (int)strlen(tail));  // "T [hh:mm:ss] [" is 14 columns
        const int fill = std::min(width, (int)(frac * width));
        std::string done((size_t)fill, '#'), rest;
        if (fill < width) {
            done += '>';
            rest.assign((size_t)(width - fill - 1), '-');
        }
        fprintf(stderr, "\r\x1b[2K\x1b[32m%s\x1b[0m [%s] [\x1b[36m%s\x1b[34m%s\x1b[0m%s", ticks[tick_++ % 8],
                hms((uint64_t)el).c_str(), done.c_str(), rest.c_str(), tail);
        fflush(stderr);
        drawn_ = true;
    }
    uint64_t len_, pos_ = 0, last_pos_ = 0, updates_ = 0;
    bool on_, drawn_ = false;
    unsigned tick_ = 0;
    std::chrono::steady_clock::time_point start_, last_;
};

// The LD pass's progress_report closure (main.rs:184-188): pb.set_position
// per completed chunk, on the calling thread (wld_progress_fn)
void on_progress(uint64_t pairs_done, void *user) { static_cast<ProgressBar *>(user)->set_position(pairs_done); }

// Rust `{:.3}` of an f32 (main.rs:76,106): exact integer rounding, tsv_format.hpp
using wld_tsv::fmt3;
using wld_tsv::fmt_u64;

struct Opt {
    std::string fasta_input, vcf_input, weights_output, pair_output;
    float min_acgt = 0.8f, min_minor = 0.02f, max_minor = 0.5f, r2_threshold = 0.1f;
    bool unweighted = false;
    bool gpu_prepass = false;
    bool exact_sums = false;  // --exact-sums: WLD_OPT_REF_SUMS 0
    int device = 0;
    std::vector<int> devices;  // --devices: a multi-device context
    int kernel = WLD_KERNEL_AUTO;
};

void usage(FILE *f) {
    fprintf(f,
            "weighted_ld 0.1.0\n"
            "A tool for computing sequence weighted linkage disequilibrium\n\n"
            "USAGE:\n    weighted_ld [FLAGS] [OPTIONS] --fasta-input <fasta-input> --pair-output <pair-output>\n\n"
            "FLAGS:\n"
            "    -h, --help          Prints help information\n"
            "        --unweighted    Use unit weights instead of Henikoff weights\n"
            "        --gpu-prepass   Filter sites and compute Henikoff weights on the GPU (FASTA input)\n"
            "        --exact-sums    (addition, not the reference's output) exact masked sums rounded once,\n"
            "                        instead of lib.rs's own f32 summation order; d' and r2 can differ from\n"
            "                        lib.rs's on rare-allele data (the default: output identical to the reference)\n"
            "    -V, --version       Prints version information\n\n"
            "OPTIONS:\n"
            "        --fasta-input <fasta-input>          The source file to load\n"
            "        --max-minor <max-minor>              Maximum fraction of minor symbols for a site to be considered "
            "[default: 0.5]\n"
            "        --min-acgt <min-acgt>                Minimum fractions of ACTG for a site to be considered "
            "[default: 0.8]\n"
            "        --min-minor <min-minor>              Minimum fraction of minor symbols for a site to be considered "
            "[default: 0.02]\n"
            "        --pair-output <pair-output>          Filename to write the per-pair weighted LD figures to, in Tab "
            "Separated Value format\n"
            "        --r2-threshold <r2-threshold>        Minimum value of R2 to be included in the output [default: "
            "0.1]\n"
            "        --weights-output <weights-output>    Filename to write the per-sequence weights to, in Tab "
            "Separated Value format\n"
            "        --vcf-input <vcf-input>              (addition) VCF input, WeightedLD.py handle_vcf semantics\n"
            "        --device <device>                    (addition) HIP device ordinal [default: 0]\n"
            "        --devices <devices>                  (addition) shard over G devices (0..G-1) or a list \"0,1,..\"\n"
            "        --kernel <kernel>                    (addition) auto | valu | mfma [default: auto]\n");
}

[[noreturn]] void arg_error(const char *msg, const char *arg) {
    fprintf(stderr, "error: %s '%s'\n\nUSAGE:\n    weighted_ld [FLAGS] [OPTIONS] --fasta-input <fasta-input> "
                    "--pair-output <pair-output>\n\nFor more information try --help\n", msg, arg);
    exit(1);
}

float parse_f32(const char *s, const char *name) {
    char *end = nullptr;
    float v = strtof(s, &end);
    if (!end || *end || !*s) {
        fprintf(stderr, "error: Invalid value for '--%s <%s>': invalid float literal\n", name, name);
        exit(1);
    }
    return v;
}

Opt parse(int argc, char **argv) {
    Opt o;
    bool have_pair = false;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i], val;
        bool has_eq = false;
        if (a.rfind("--", 0) == 0) {
            size_t eq = a.find('=');
            if (eq != std::string::npos) {
                val = a.substr(eq + 1);
                a = a.substr(0, eq);
                has_eq = true;
            }
        }
        auto need = [&](const char *name) -> std::string {
            if (has_eq) return val;
            if (i + 1 >= argc) arg_error("The argument requires a value but none was supplied:", name);
            return argv[++i];
        };
        if (a == "-h" || a == "--help") {
            usage(stdout);
            exit(0);
        } else if (a == "-V" || a == "--version") {
            printf("weighted_ld 0.1.0 (%s)\n", wld_version());
            exit(0);
        } else if (a == "--fasta-input") {
            o.fasta_input = need("--fasta-input");
        } else if (a == "--vcf-input") {
            o.vcf_input = need("--vcf-input");
        } else if (a == "--min-acgt") {
            o.min_acgt = parse_f32(need("--min-acgt").c_str(), "min-acgt");
        } else if (a == "--min-minor") {
            o.min_minor = parse_f32(need("--min-minor").c_str(), "min-minor");
        } else if (a == "--max-minor") {
            o.max_minor = parse_f32(need("--max-minor").c_str(), "max-minor");
        } else if (a == "--r2-threshold") {
            o.r2_threshold = parse_f32(need("--r2-threshold").c_str(), "r2-threshold");
        } else if (a == "--weights-output") {
            o.weights_output = need("--weights-output");
        } else if (a == "--pair-output") {
            o.pair_output = need("--pair-output");
            have_pair = true;
        } else if (a == "--unweighted") {
            o.unweighted = true;
        } else if (a == "--exact-sums") {
            o.exact_sums = true;
        } else if (a == "--gpu-prepass") {
            o.gpu_prepass = true;
        } else if (a == "--device") {
            o.device = atoi(need("--device").c_str());
        } else if (a == "--devices") {
            const std::string v = need("--devices");
            o.devices.clear();
            if (v.find(',') == std::string::npos) {
                const int g = atoi(v.c_str());
                if (g < 1) arg_error("Invalid value for '--devices':", v.c_str());
                for (int k = 0; k < g; ++k) o.devices.push_back(k);
            } else {
                size_t at = 0;
                while (at <= v.size()) {
                    const size_t e = std::min(v.find(',', at), v.size());
                    const std::string t = v.substr(at, e - at);
                    if (t.empty() || t.find_first_not_of("0123456789") != std::string::npos)
                        arg_error("Invalid value for '--devices':", v.c_str());
                    o.devices.push_back(atoi(t.c_str()));
                    at = e + 1;
                }
            }
        } else if (a == "--kernel") {
            std::string k = need("--kernel");
            o.kernel = k == "valu" ? WLD_KERNEL_VALU : k == "mfma" ? WLD_KERNEL_MFMA : WLD_KERNEL_AUTO;
            if (k != "valu" && k != "mfma" && k != "auto") arg_error("Invalid value for '--kernel':", k.c_str());
        } else {
            arg_error("Found argument which wasn't expected, or isn't valid in this context:", argv[i]);
        }
    }
    if (o.fasta_input.empty() && o.vcf_input.empty())
        arg_error("The following required arguments were not provided:", "--fasta-input <fasta-input>");
    if (!have_pair) arg_error("The following required arguments were not provided:", "--pair-output <pair-output>");
    if (o.gpu_prepass && o.devices.size() > 1)
        arg_error("The argument '--gpu-prepass' cannot be used with", "--devices (the device pre-pass runs on one device)");
    return o;
}

// Ends the process from any point after the device-context thread started:
// streams are flushed, but no static destructor runs — the HIP runtime may
// still be starting up on that thread, and tearing it down underneath it
// crashes (SIGSEGV seen on the GPU box).  A Rust panic likewise just ends the
// process with the other threads still running.
[[noreturn]] void quit(int code) {
    fflush(nullptr);
    _exit(code);
}

// Rust's `main() -> Result<(), io::Error>` prints "Error: ..." and exits 1;
// a panic prints the panic message and exits 101.
// msg: the failed call's wld_last_error() (thread-local: pass it when the call
// ran on another thread).
[[noreturn]] void die(int st, const char *what, const char *msg = nullptr) {
    if (!msg) msg = wld_last_error();
    if (st == WLD_E_FORMAT || st == WLD_E_ARG) {
        fprintf(stderr, "thread 'main' panicked at '%s: %s'\n", what, msg);
        quit(101);
    }
    fprintf(stderr, "Error: %s: %s (%s)\n", what, wld_status_string(st), msg);
    quit(1);
}

std::string debug_path(const std::string &p) { return "\"" + p + "\""; }

// main.rs:70-80
int write_henikoff_weights(const std::string &path, const std::vector<float> &w) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return WLD_E_IO;
    std::string out = "Sequence_index\thk_weight\n";
    char buf[64];
    for (size_t i = 0; i < w.size(); ++i) {
        int n = fmt_u64(buf, i);
        buf[n++] = '\t';
        n += fmt3(buf + n, w[i]);
        buf[n++] = '\n';
        out.append(buf, n);
    }
    size_t ok = fwrite(out.data(), 1, out.size(), f);
    int rc = fclose(f);
    return (ok == out.size() && rc == 0) ? WLD_OK : WLD_E_IO;
}

// main.rs:82-119: header, then "{}\t{}\t{:.3}\t{:.3}\t{:.3}" per row in PairStore order.
// Worker threads claim blocks of rows in order and format them into a ring of
// slot buffers; the calling thread writes finished blocks in order, so
// formatting overlaps the file write and memory stays at 2 slots per worker.
int write_pair_stats(const std::string &path, const wld_pairs &p) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return WLD_E_IO;
    const char *hdr = "site_a\tsite_b\td\td'\tr2\n";
    bool ok = fwrite(hdr, 1, strlen(hdr), f) == strlen(hdr);
    const uint64_t n = p.n, block = 1 << 16;
    const uint64_t n_blocks = (n + block - 1) / block;
    ProgressBar pb(n);  // main.rs:89-97: set_position every 5000 rows written (main.rs:111-116)
    const unsigned nt =
        (unsigned)std::max<uint64_t>(1, std::min<uint64_t>({std::thread::hardware_concurrency(), 32, n_blocks}));
    const uint64_t n_slots = 2 * (uint64_t)nt;
    struct Slot {
        std::vector<char> buf;
        size_t len = 0;
        uint64_t ready = UINT64_MAX;  // block index whose text the slot holds
    };
    std::vector<Slot> slots(n_slots);
    std::mutex mu;
    std::condition_variable cv_ready, cv_free;
    uint64_t next_claim = 0, next_write = 0;
    bool abort = false;
    auto worker = [&] {
        for (;;) {
            uint64_t b;
            {
                std::unique_lock<std::mutex> lk(mu);
                if (next_claim >= n_blocks || abort) return;
                b = next_claim++;
                // slot b % n_slots is free once block b - n_slots has been written
                cv_free.wait(lk, [&] { return abort || next_write + n_slots > b; });
                if (abort) return;
            }
            Slot &sl = slots[b % n_slots];
            const uint64_t lo = b * block, hi = std::min(n, lo + block);
            if (sl.buf.size() < (hi - lo) * 48) sl.buf.resize((hi - lo) * 48);
            size_t k = 0;
            for (uint64_t i = lo; i < hi; ++i) {
                if (k + 256 > sl.buf.size()) sl.buf.resize(sl.buf.size() * 2);
                char *o = sl.buf.data() + k;
                int m = fmt_u64(o, p.site_a[i]);
                o[m++] = '\t';
                m += fmt_u64(o + m, p.site_b[i]);
                o[m++] = '\t';
                m += fmt3(o + m, p.d[i]);
                o[m++] = '\t';
                m += fmt3(o + m, p.d_prime[i]);
                o[m++] = '\t';
                m += fmt3(o + m, p.r2[i]);
                o[m++] = '\n';
                k += m;
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                sl.len = k;
                sl.ready = b;
            }
            cv_ready.notify_all();
        }
    };
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt && n_blocks; ++t) th.emplace_back(worker);
    for (uint64_t b = 0; b < n_blocks; ++b) {
        Slot &sl = slots[b % n_slots];
        {
            std::unique_lock<std::mutex> lk(mu);
            cv_ready.wait(lk, [&] { return sl.ready == b; });
        }
        if (ok && fwrite(sl.buf.data(), 1, sl.len, f) != sl.len) ok = false;
        const uint64_t written = std::min(n, (b + 1) * block);
        if (written / 5000 > b * block / 5000) pb.set_position(written / 5000 * 5000);
        {
            std::lock_guard<std::mutex> lk(mu);
            sl.ready = UINT64_MAX;
            ++next_write;
            if (!ok) abort = true;
        }
        cv_free.notify_all();
        if (!ok) break;
    }
    for (auto &x : th) x.join();
    if (fclose(f) != 0) ok = false;
    return ok ? WLD_OK : WLD_E_IO;
}

// (debug level only, so info-level output is the reference's: the LD pass's
// progress_report calls — progress(0), then one per 256x256 chunk)
void log_progress(const ProgressBar &pb) {
    log_at(4, "progress: %" PRIu64 " progress_report calls, last %" PRIu64 " pairs", pb.updates(),
           pb.last_position());
}

// main.rs:186-212 after the pair computation: timing logs, TSV, clean-up.
int finish(const Opt &opt, wld_ctx *ctx, wld_pairs &pairs, std::chrono::steady_clock::duration dur,
           uint64_t total_pairs) {
    using clk = std::chrono::steady_clock;
    INFO("Finished computing pairwise weighted LD stats in %s", fmt_duration(dur).c_str());
    const double secs = std::chrono::duration<double>(dur).count();
    INFO("    %s pairs computed at ~%s, %s passed threshold", human((double)total_pairs).c_str(),
         human((double)total_pairs / secs, "pairs/s").c_str(), human((double)pairs.n).c_str());
    wld_run_stats rs;
    if (wld_last_stats(ctx, &rs) == WLD_OK)
        log_at(4, "device: kernel=%s pairs=%" PRIu64 " pair_kernel=%.3fms order=%.3fms",
               rs.kernel == WLD_KERNEL_MFMA ? "mfma" : "valu", rs.pairs, rs.pair_kernel_ms, rs.order_ms);

    INFO("Writing output to %s", debug_path(opt.pair_output).c_str());
    auto sw = clk::now();
    if (write_pair_stats(opt.pair_output, pairs) != WLD_OK) {
        fprintf(stderr, "Error: cannot write %s\n", opt.pair_output.c_str());
        return 1;
    }
    INFO("Finshed writing output in %s", fmt_duration(clk::now() - sw).c_str());  // (sic) main.rs:210
    wld_pairs_free(&pairs);
    wld_destroy(ctx);
    return 0;
}

// --gpu-prepass: main.rs:139-190 with the site filter and Henikoff weights on
// the device (wld_load_filtered), then the staged run and a host copy of the rows.
int run_gpu_prepass(const Opt &opt, wld_siteset *siteset, wld_ctx *ctx) {
    using clk = std::chrono::steady_clock;
    const size_t L0 = wld_siteset_n_sites(siteset), N = wld_siteset_n_seqs(siteset);
    auto sw = clk::now();
    size_t L = 0;
    int st = wld_load_filtered(ctx, wld_siteset_buffer(siteset), L0, N, wld_siteset_site_map(siteset), opt.min_acgt,
                               opt.min_minor, opt.max_minor, opt.unweighted ? 1 : 0, &L);
    if (st != WLD_OK) die(st, "load_filtered");
    INFO("Computed + filtered sites of interest%s on the GPU in %s", opt.unweighted ? "" : " and Henikoff weights",
         fmt_duration(clk::now() - sw).c_str());
    INFO("    Found %zu sites of interest", L);
    if (!opt.weights_output.empty()) {
        std::vector<float> weights(N);
        if ((st = wld_weights_copy(ctx, weights.data())) != WLD_OK) die(st, "weights_copy");
        INFO("Writing weights to %s", debug_path(opt.weights_output).c_str());
        if (write_henikoff_weights(opt.weights_output, weights) != WLD_OK) {
            fprintf(stderr, "Error: cannot write %s\n", opt.weights_output.c_str());
            quit(1);  // the context thread may still be running
        }
    }
    INFO("Beginning pairwise weighted LD computation");
    sw = clk::now();
    const uint64_t total_pairs = ((uint64_t)L - 1) * ((uint64_t)L - 2) / 2;  // main.rs:168 (sic, wraps)
    wld_pairs pairs;  // any L: batches of <= 2^31 pairs, rows appended in reference order
    {
        ProgressBar pb(total_pairs);  // main.rs:170-178
        on_progress(0, &pb);  // all_weighted_ld_pairs' initial report (lib.rs:584); wld_run_host reports chunks only
        if ((st = wld_run_host(ctx, opt.r2_threshold, on_progress, &pb, &pairs)) != WLD_OK)
            die(st, "all_weighted_ld_pairs");
        log_progress(pb);
    }
    return finish(opt, ctx, pairs, clk::now() - sw, total_pairs);
}

}  // namespace

int main(int argc, char **argv) {
    init_logger();
    Opt opt = parse(argc, argv);
    using clk = std::chrono::steady_clock;
    if (opt.exact_sums) {
        // not a reference flag (main.rs:14-68 has none like it): printed at any
        // log level, since the TSV it produces is not lib.rs's
        const int keep = g_level;
        g_level = std::max(g_level, 2);
        log_at(2, "--exact-sums departs from the reference: the masked sums are exact sums rounded once, not "
                  "lib.rs's f32 summation order, so d, d' and r2 differ from lib.rs's where its own f32 rounding "
                  "shows (measured on rare-allele data: |d'| up to 1.11, |r2| up to 0.023 against lib.rs); "
                  "without the flag the output is lib.rs's, bit for bit");
        g_level = keep;
    }

    // The device context (HIP runtime start-up) is created while the input is
    // read, so that the LD timing below covers the computation only.
    wld_ctx *ctx = nullptr;
    int ctx_st = WLD_OK;
    std::string ctx_msg;
    std::thread ctx_thread([&] {
        ctx_st = opt.devices.empty() ? wld_create(opt.device, &ctx)
                                     : wld_create_multi(opt.devices.data(), (int)opt.devices.size(), &ctx);
        if (ctx_st != WLD_OK) ctx_msg = wld_last_error();
    });
    auto get_ctx = [&]() -> wld_ctx * {
        if (ctx_thread.joinable()) ctx_thread.join();
        if (ctx_st != WLD_OK) die(ctx_st, "wld_create", ctx_msg.c_str());
        if (opt.kernel != WLD_KERNEL_AUTO) {
            int s2 = wld_set_kernel(ctx, opt.kernel);
            if (s2 != WLD_OK) die(s2, "wld_set_kernel");
        }
        if (opt.exact_sums) {
            int s2 = wld_set_option(ctx, WLD_OPT_REF_SUMS, 0);
            if (s2 != WLD_OK) die(s2, "wld_set_option");
        }
        return ctx;
    };

    auto sw = clk::now();
    wld_siteset *siteset = nullptr;
    int st;
    const bool vcf = !opt.vcf_input.empty();
    if (vcf)
        st = wld_read_vcf(opt.vcf_input.c_str(), &siteset);
    else
        st = wld_read_fasta(opt.fasta_input.c_str(), &siteset);
    if (st != WLD_OK) die(st, vcf ? "read_vcf" : "read_fasta");
    INFO("Loaded %s file in %s", vcf ? "vcf" : "fasta", fmt_duration(clk::now() - sw).c_str());
    INFO("    %zu sequences, %zu sites", wld_siteset_n_seqs(siteset), wld_siteset_n_sites(siteset));

    if (opt.gpu_prepass && !vcf) return run_gpu_prepass(opt, siteset, get_ctx());

    sw = clk::now();
    wld_siteset *filtered = nullptr;
    if (vcf) {
        // handle_vcf has no variable-site filter (WeightedLD.py:382-402)
        filtered = siteset;
        siteset = nullptr;
        INFO("VCF input: no site filter (WeightedLD.py handle_vcf semantics)");
    } else {
        st = wld_siteset_filter_sites_of_interest(siteset, opt.min_acgt, opt.min_minor, opt.max_minor, &filtered);
        if (st != WLD_OK) die(st, "filter_by");
        INFO("Computed + filtered sites of interest in %s", fmt_duration(clk::now() - sw).c_str());
    }
    const size_t L = wld_siteset_n_sites(filtered), N = wld_siteset_n_seqs(filtered);
    INFO("    Found %zu sites of interest", L);

    std::vector<float> weights(N, 1.0f);
    if (!opt.unweighted) {
        sw = clk::now();
        st = wld_henikoff_weights(filtered, weights.data());
        if (st != WLD_OK) die(st, "henikoff_weights");
        INFO("Computed Henikoff weights in %s", fmt_duration(clk::now() - sw).c_str());
    }
    if (!opt.weights_output.empty()) {
        INFO("Writing weights to %s", debug_path(opt.weights_output).c_str());
        if (write_henikoff_weights(opt.weights_output, weights) != WLD_OK) {
            fprintf(stderr, "Error: cannot write %s\n", opt.weights_output.c_str());
            quit(1);  // the context thread may still be running
        }
    }

    INFO("Beginning pairwise weighted LD computation");
    sw = clk::now();
    const uint64_t total_pairs = ((uint64_t)L - 1) * ((uint64_t)L - 2) / 2;  // main.rs:168 (sic, wraps)
    get_ctx();
    wld_pairs pairs;
    {
        ProgressBar pb(total_pairs);  // main.rs:170-178, fed by the closure of main.rs:184-188
        st = wld_all_weighted_ld_pairs(ctx, wld_siteset_buffer(filtered), L, N, wld_siteset_site_map(filtered),
                                       weights.data(), opt.r2_threshold, on_progress, &pb, &pairs);
        if (st != WLD_OK) die(st, "all_weighted_ld_pairs");
        log_progress(pb);
    }
    const int rc = finish(opt, ctx, pairs, clk::now() - sw, total_pairs);
    wld_siteset_free(filtered);
    wld_siteset_free(siteset);
    return rc;
}
