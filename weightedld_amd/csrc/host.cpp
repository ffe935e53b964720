// Host pre-pass of the WeightedLD pipeline (north_star: FASTA -> int matrix,
// variable-site masks and Henikoff weights stay on the host).
//
// Restates, in C++ for the library the CLI and the Python mirror share:
//   Symbol / From<char>          lib.rs:20-64
//   SymbolHistogram              lib.rs:72-141
//   SiteSet (+ filter_by)        lib.rs:158-275
//   read_fasta                   lib.rs:277-307
//   is_site_of_interest          lib.rs:309-338
//   henikoff_weights             lib.rs:340-380
//   handle_vcf (Python)          WeightedLD.py:311-379
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cctype>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <array>
#include <thread>

#include "common.hpp"

namespace wld {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

void clear_error() { g_err.clear(); }

int fail(int status, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return status;
}

// lib.rs:98-104 (bytes >= 6 count as Unknown, 5).  One vectorisable compare-
// and-count pass per symbol value over blocks of 255 bytes (u8 counters).
void histogram(const uint8_t *sym, size_t n, uint64_t out[6]) {
    uint64_t h[5] = {0, 0, 0, 0, 0};
    for (size_t i0 = 0; i0 < n; i0 += 255) {
        const size_t m = std::min<size_t>(255, n - i0);
        for (int v = 0; v < 5; ++v) {
            uint8_t c = 0;
            for (size_t i = 0; i < m; ++i) c += sym[i0 + i] == v;
            h[v] += c;
        }
    }
    uint64_t known = 0;
    for (int s = 0; s < 5; ++s) {
        out[s] = h[s];
        known += h[s];
    }
    out[5] = n - known;
}

// lib.rs:126-140: strict '>' keeps the earlier of A,C,G,T,- on ties.
void major_minor(const uint64_t h[6], int *maj, int *mnr) {
    int a = WLD_NONE, b = WLD_NONE;
    for (int s = WLD_SYM_A; s <= WLD_SYM_MISSING; ++s) {
        uint64_t ca = a >= 0 ? h[a] : 0, cb = b >= 0 ? h[b] : 0;
        if (h[s] > ca) {
            b = a;
            a = s;
        } else if (h[s] > cb) {
            b = s;
        }
    }
    *maj = a;
    *mnr = b;
}

// f(lo, hi) over [0, n) split across the host threads; serial below min_n items.
template <class F>
static void parallel_for(size_t n, F &&f, size_t min_n = 4096) {
    unsigned nt = std::max(1u, std::min(std::thread::hardware_concurrency(), 64u));
    if (n < min_n || nt == 1) {
        f(size_t(0), n);
        return;
    }
    std::vector<std::thread> th;
    size_t step = (n + nt - 1) / nt;
    for (unsigned t = 0; t < nt; ++t) {
        size_t lo = t * step, hi = std::min(n, lo + step);
        if (lo >= hi) break;
        th.emplace_back([&f, lo, hi] { f(lo, hi); });
    }
    for (auto &x : th) x.join();
}

void compute_histograms(SiteSet &s) {
    s.hist.assign(s.n_sites * 6, 0);
    parallel_for(s.n_sites, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) histogram(&s.buffer[i * s.n_seqs], s.n_seqs, &s.hist[i * 6]);
    });
}

// lib.rs:53-64, as a table for the FASTA transpose
static const std::array<uint8_t, 256> kSymbolOfByte = [] {
    std::array<uint8_t, 256> t{};
    for (int c = 0; c < 256; ++c) t[c] = WLD_SYM_UNKNOWN;
    t['a'] = t['A'] = WLD_SYM_A;
    t['c'] = t['C'] = WLD_SYM_C;
    t['g'] = t['G'] = WLD_SYM_G;
    t['t'] = t['T'] = WLD_SYM_T;
    t['-'] = WLD_SYM_MISSING;
    return t;
}();

// lib.rs:53-64
static inline uint8_t symbol_from_byte(unsigned char c) {
    switch (c) {
    case 'a': case 'A': return WLD_SYM_A;
    case 'c': case 'C': return WLD_SYM_C;
    case 'g': case 'G': return WLD_SYM_G;
    case 't': case 'T': return WLD_SYM_T;
    case '-': return WLD_SYM_MISSING;
    default: return WLD_SYM_UNKNOWN;
    }
}

// The whole file, memory-mapped read-only (falls back to read_file).
struct FileView {
    const unsigned char *p = nullptr;
    size_t n = 0;
    void *map = nullptr;
    std::string copy;
    ~FileView() {
        if (map) munmap(map, n);
    }
};

static bool read_file(const char *path, std::string &data);

static bool view_file(const char *path, FileView &v) {
    const int fd = open(path, O_RDONLY);
    if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0) {
            void *m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
            if (m != MAP_FAILED) {
                close(fd);
                v.map = m;
                v.p = (const unsigned char *)m;
                v.n = (size_t)st.st_size;
                return true;
            }
        }
        close(fd);
    }
    if (!read_file(path, v.copy)) return false;
    v.p = (const unsigned char *)v.copy.data();
    v.n = v.copy.size();
    return true;
}

static bool read_file(const char *path, std::string &data) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return false; }
    long sz = ftell(f);
    if (sz < 0) { fclose(f); return false; }
    fseek(f, 0, SEEK_SET);
    data.resize((size_t)sz);
    size_t got = sz ? fread(&data[0], 1, (size_t)sz, f) : 0;
    fclose(f);
    data.resize(got);
    return true;
}

// Number of UTF-8 chars (what Rust's str::chars() yields) in [p, p+n).
static size_t utf8_chars(const unsigned char *p, size_t n) {
    size_t c = 0;
    for (size_t i = 0; i < n; ++i) c += (p[i] & 0xC0) != 0x80;
    return c;
}

}  // namespace wld

using namespace wld;

extern "C" {

const char *wld_last_error(void) { return g_err.c_str(); }

const char *wld_status_string(int st) {
    switch (st) {
    case WLD_OK: return "ok";
    case WLD_E_ARG: return "invalid argument";
    case WLD_E_HIP: return "HIP runtime error";
    case WLD_E_OOM: return "out of memory";
    case WLD_E_NODEV: return "no gfx950 device";
    case WLD_E_IO: return "I/O error";
    case WLD_E_FORMAT: return "input format error";
    case WLD_E_STATE: return "invalid call order";
    default: return "unknown status";
    }
}

int wld_histogram(const uint8_t *symbols, size_t n, uint64_t out[6]) {
    if ((!symbols && n) || !out) return fail(WLD_E_ARG, "wld_histogram: null pointer");
    histogram(symbols, n, out);
    return WLD_OK;
}

int wld_major_minor(const uint64_t hist[6], int *major, int *minor) {
    if (!hist || !major || !minor) return fail(WLD_E_ARG, "wld_major_minor: null pointer");
    major_minor(hist, major, minor);
    return WLD_OK;
}

// lib.rs:277-307 then SiteSet::from_multiseq (lib.rs:176-206).
int wld_read_fasta(const char *path, wld_siteset **out) {
    if (!path || !out) return fail(WLD_E_ARG, "wld_read_fasta: null pointer");
    FileView view;
    if (!view_file(path, view)) return fail(WLD_E_IO, "cannot read %s", path);
    const unsigned char *p = view.p;
    const size_t n = view.n;
    std::vector<size_t> start, bytes;
    bool any_high = false;
    for (size_t pos = 0; pos < n;) {
        const void *nl = memchr(p + pos, '\n', n - pos);
        size_t e = nl ? (size_t)((const unsigned char *)nl - p) + 1 : n;  // keep '\n'
        if (p[pos] != '>') {
            start.push_back(pos);
            bytes.push_back(e - pos);
        }
        pos = e;
    }
    if (start.empty())
        return fail(WLD_E_FORMAT, "%s: no sequences (the reference indexes sequences[0] and panics)", path);
    {  // any byte >= 0x80 (then multi-byte UTF-8 chars count as one symbol each)
        uint64_t acc = 0, w;
        size_t i = 0;
        for (; i + 8 <= n; i += 8) {
            memcpy(&w, p + i, 8);
            acc |= w;
        }
        for (; i < n; ++i) acc |= p[i];
        any_high = (acc & 0x8080808080808080ull) != 0;
    }

    auto *ss = new wld_siteset;
    SiteSet &s = ss->s;
    s.n_seqs = start.size();
    if (!any_high) {
        s.n_sites = bytes[0];
        for (size_t i = 0; i < start.size(); ++i)
            if (bytes[i] != s.n_sites) {
                const size_t n0 = s.n_sites;  // s lives in ss
                delete ss;
                return fail(WLD_E_FORMAT,
                            "%s: Not all sequences have the same number of symbols (sequence %zu has %zu, "
                            "sequence 0 has %zu; lib.rs:180-182)", path, i, bytes[i], n0);
            }
        s.buffer.resize(s.n_sites * s.n_seqs);
        s.hist.resize(s.n_sites * 6);
        // cache-blocked transpose into site-major order, threads over 64-site
        // blocks: each 64x64 tile is gathered from 64 lines into a local tile,
        // then written as 64 contiguous runs of the site-major rows; the
        // block's histograms are taken while its rows are still in cache
        const size_t B = 64, N = s.n_seqs;
        uint8_t *dst = s.buffer.data();
        parallel_for((s.n_sites + B - 1) / B, [&](size_t lo, size_t hi) {
            alignas(64) uint8_t tile[B][B];
            for (size_t jb = lo; jb < hi; ++jb) {
                const size_t j0 = jb * B, nj = std::min(s.n_sites, j0 + B) - j0;
                for (size_t q0 = 0; q0 < N; q0 += B) {
                    const size_t nq = std::min(N, q0 + B) - q0;
                    for (size_t q = 0; q < nq; ++q) {
                        const unsigned char *line = p + start[q0 + q] + j0;
                        for (size_t j = 0; j < nj; ++j) tile[j][q] = kSymbolOfByte[line[j]];
                    }
                    for (size_t j = 0; j < nj; ++j) memcpy(dst + (j0 + j) * N + q0, tile[j], nq);
                }
                for (size_t j = 0; j < nj; ++j) histogram(dst + (j0 + j) * N, N, &s.hist[(j0 + j) * 6]);
            }
        }, 2);
    } else {
        // Slow path: multi-byte UTF-8 chars are one (Unknown) symbol each.
        std::vector<size_t> chars(start.size());
        for (size_t i = 0; i < start.size(); ++i) chars[i] = utf8_chars(p + start[i], bytes[i]);
        s.n_sites = chars[0];
        for (size_t i = 0; i < start.size(); ++i)
            if (chars[i] != s.n_sites) {
                delete ss;
                return fail(WLD_E_FORMAT, "%s: Not all sequences have the same number of symbols", path);
            }
        s.buffer.resize(s.n_sites * s.n_seqs);
        for (size_t q = 0; q < s.n_seqs; ++q) {
            size_t j = 0;
            for (size_t k = 0; k < bytes[q]; ++k) {
                unsigned char c = p[start[q] + k];
                if ((c & 0xC0) == 0x80) continue;
                s.buffer[j++ * s.n_seqs + q] = symbol_from_byte(c);
            }
        }
        compute_histograms(s);
    }
    *out = ss;
    return WLD_OK;
}

int wld_siteset_from_buffer(const uint8_t *site_major, size_t n_sites, size_t n_seqs,
                            const uint64_t *site_map, wld_siteset **out) {
    if (!out || (!site_major && n_sites && n_seqs)) return fail(WLD_E_ARG, "wld_siteset_from_buffer: null pointer");
    auto *ss = new wld_siteset;
    SiteSet &s = ss->s;
    s.n_sites = n_sites;
    s.n_seqs = n_seqs;
    s.buffer.assign(site_major, site_major + n_sites * n_seqs);
    for (auto &b : s.buffer)
        if (b > WLD_SYM_UNKNOWN) b = WLD_SYM_UNKNOWN;
    if (site_map) {
        s.has_map = true;
        s.site_map.assign(site_map, site_map + n_sites);
    }
    compute_histograms(s);
    *out = ss;
    return WLD_OK;
}

void wld_siteset_free(wld_siteset *s) { delete s; }
size_t wld_siteset_n_sites(const wld_siteset *s) { return s ? s->s.n_sites : 0; }
size_t wld_siteset_n_seqs(const wld_siteset *s) { return s ? s->s.n_seqs : 0; }
const uint8_t *wld_siteset_buffer(const wld_siteset *s) { return s && !s->s.buffer.empty() ? s->s.buffer.data() : nullptr; }
const uint64_t *wld_siteset_site_map(const wld_siteset *s) { return s && s->s.has_map ? s->s.site_map.data() : nullptr; }
uint64_t wld_siteset_parent_site_index(const wld_siteset *s, size_t i) {
    return s->s.has_map ? s->s.site_map[i] : (uint64_t)i;
}
int wld_siteset_histogram(const wld_siteset *s, size_t site, uint64_t out[6]) {
    if (!s || !out || site >= s->s.n_sites) return fail(WLD_E_ARG, "wld_siteset_histogram: bad site");
    for (int k = 0; k < 6; ++k) out[k] = s->s.hist[site * 6 + k];
    return WLD_OK;
}

// lib.rs:309-338
int wld_is_site_of_interest(const uint8_t *site, size_t n, size_t min_acgt, float min_minor, float max_minor) {
    uint64_t h[6];
    histogram(site, n, h);
    uint64_t acgt = h[0] + h[1] + h[2] + h[3];
    if (acgt <= min_acgt) return 0;
    int maj, mnr;
    major_minor(h, &maj, &mnr);
    if (maj < 0 || mnr < 0) return 0;
    float maj_count = (float)h[maj], min_count = (float)h[mnr];
    float minor_frac = min_count / (min_count + maj_count);
    return !(minor_frac < min_minor || minor_frac > max_minor);
}

// main.rs:139-143 + SiteSet::filter_by (lib.rs:230-251).  The histogram of a
// kept site is the parent's (lib.rs:240), i.e. is_site_of_interest's own.
int wld_siteset_filter_sites_of_interest(const wld_siteset *in, float min_acgt_frac, float min_minor,
                                         float max_minor, wld_siteset **out) {
    if (!in || !out) return fail(WLD_E_ARG, "wld_siteset_filter_sites_of_interest: null pointer");
    const SiteSet &s = in->s;
    float c = std::ceil(min_acgt_frac * (float)s.n_seqs);
    size_t min_acgt = c <= 0.0f ? 0 : (size_t)c;  // Rust `as usize` saturates at 0
    auto *o = new wld_siteset;
    SiteSet &t = o->s;
    t.n_seqs = s.n_seqs;
    t.has_map = true;  // filter_by always records a site_map (lib.rs:248)
    for (size_t i = 0; i < s.n_sites; ++i) {
        const uint64_t *h = &s.hist[i * 6];
        uint64_t acgt = h[0] + h[1] + h[2] + h[3];
        bool keep = false;
        if (acgt > min_acgt) {
            int maj, mnr;
            major_minor(h, &maj, &mnr);
            if (maj >= 0 && mnr >= 0) {
                float mj = (float)h[maj], mn = (float)h[mnr];
                float frac = mn / (mn + mj);
                keep = !(frac < min_minor || frac > max_minor);
            }
        }
        if (keep) t.site_map.push_back(i);
    }
    t.n_sites = t.site_map.size();
    t.buffer.resize(t.n_sites * t.n_seqs);
    t.hist.resize(t.n_sites * 6);
    parallel_for(t.n_sites, [&](size_t lo, size_t hi) {
        for (size_t k = lo; k < hi; ++k) {
            size_t i = t.site_map[k];
            memcpy(&t.buffer[k * t.n_seqs], &s.buffer[i * s.n_seqs], s.n_seqs);
            memcpy(&t.hist[k * 6], &s.hist[i * 6], 6 * sizeof(uint64_t));
        }
    }, 256);
    *out = o;
    return WLD_OK;
}

// lib.rs:340-380.  Bit-for-bit the reference's f32 order: per site, the
// contribution 1/(distinct*count) and the running site total (sequential over
// sequences, lib.rs:366-371); per sequence, contributions summed over sites in
// order (ndarray sum_axis(Axis(0)) on a non-contiguous axis); divide by the
// max folded from 0.0 with f32::max.
int wld_henikoff_weights(const wld_siteset *in, float *out) {
    if (!in || !out) return fail(WLD_E_ARG, "wld_henikoff_weights: null pointer");
    const SiteSet &s = in->s;
    const size_t L = s.n_sites, N = s.n_seqs;
    // per-site: contribution per symbol (index 0..4) and the Unknown fill (index 5)
    std::vector<float> tab(L * 6);
    parallel_for(L, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            const uint64_t *h = &s.hist[i * 6];
            size_t distinct = 0;
            for (int k = 0; k <= WLD_SYM_MISSING; ++k) distinct += h[k] > 0;
            float df = (float)distinct;
            float c[6];
            for (int k = 0; k <= WLD_SYM_MISSING; ++k) c[k] = 1.0f / (df * (float)h[k]);
            // the Unknown fill is read only by sequences that are Unknown here
            float total = 0.0f;
            if (h[5]) {
                const uint8_t *site = &s.buffer[i * N];
                for (size_t q = 0; q < N; ++q)
                    if (site[q] <= WLD_SYM_MISSING) total += c[site[q]];
            }
            c[5] = total / df;
            for (int k = 0; k < 6; ++k) tab[i * 6 + k] = c[k];
        }
    });
    std::vector<float> w(N, 0.0f);
    parallel_for(N, [&](size_t lo, size_t hi) {
        for (size_t i = 0; i < L; ++i) {
            const uint8_t *site = &s.buffer[i * N];
            const float *c = &tab[i * 6];
            for (size_t q = lo; q < hi; ++q) w[q] = w[q] + c[site[q]];
        }
    }, 64);
    float mx = 0.0f;
    for (size_t q = 0; q < N; ++q) mx = std::fmax(mx, w[q]);
    for (size_t q = 0; q < N; ++q) out[q] = w[q] / mx;
    return WLD_OK;
}

// ---------------------------------------------------------------- VCF
// WeightedLD.py:311-379, string transforms restated without a regex engine.
static std::string replace_all(const std::string &t, const std::string &from, const std::string &to) {
    std::string r;
    r.reserve(t.size());
    size_t i = 0;
    while (i < t.size()) {
        if (t.compare(i, from.size(), from) == 0) {
            r += to;
            i += from.size();
        } else {
            r += t[i++];
        }
    }
    return r;
}

static inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

// re.sub(r"[^0-9]\|[^0-9]", "", t): non-overlapping, left to right
static std::string drop_nondigit_pipe_nondigit(const std::string &t) {
    std::string r;
    r.reserve(t.size());
    size_t i = 0;
    while (i < t.size()) {
        if (i + 2 < t.size() && !is_digit(t[i]) && t[i + 1] == '|' && !is_digit(t[i + 2])) {
            i += 3;
        } else {
            r += t[i++];
        }
    }
    return r;
}

// re.sub(r"./.", ".|.", t): '.' is any char but '\n'
static std::string unphased_to_missing(const std::string &t) {
    std::string r;
    r.reserve(t.size());
    size_t i = 0;
    while (i < t.size()) {
        if (i + 2 < t.size() && t[i] != '\n' && t[i + 1] == '/' && t[i + 2] != '\n') {
            r += ".|.";
            i += 3;
        } else {
            r += t[i++];
        }
    }
    return r;
}

static bool parse_int(const std::string &f, long long &v) {
    // numpy str -> int64 conversion (Python int(): surrounding whitespace ok)
    size_t a = 0, b = f.size();
    while (a < b && isspace((unsigned char)f[a])) ++a;
    while (b > a && isspace((unsigned char)f[b - 1])) --b;
    if (a == b) return false;
    std::string s = f.substr(a, b - a);
    std::string digits;
    for (char c : s)
        if (c != '_') digits += c;
    char *end = nullptr;
    errno = 0;
    v = strtoll(digits.c_str(), &end, 10);
    return errno == 0 && end && *end == 0;
}

int wld_read_vcf(const char *path, wld_siteset **out) {
    if (!path || !out) return fail(WLD_E_ARG, "wld_read_vcf: null pointer");
    std::string data;
    if (!read_file(path, data)) return fail(WLD_E_IO, "cannot read %s", path);
    std::vector<std::string> lines;
    {
        size_t pos = 0;
        for (;;) {
            size_t e = data.find('\n', pos);
            if (e == std::string::npos) {
                lines.push_back(data.substr(pos));
                break;
            }
            lines.push_back(data.substr(pos, e - pos));
            pos = e + 1;
        }
    }
    size_t hdr = lines.size();
    for (size_t i = 0; i < lines.size(); ++i)
        if (lines[i].find("#CHROM") != std::string::npos) { hdr = i; break; }
    if (hdr == lines.size()) return fail(WLD_E_FORMAT, "No #CHROM header block identified");
    std::vector<std::string> rows(lines.begin() + hdr + 1, lines.end());
    if (rows.empty()) return fail(WLD_E_FORMAT, "%s: no data lines after #CHROM", path);
    {
        size_t ncol = 1;
        for (char c : rows[0]) ncol += c == '\t';
        if (ncol <= 12)
            return fail(WLD_E_FORMAT, "The VCF data contains too small a population, are you sure this is a multi VCF?");
    }
    std::vector<std::vector<std::string>> fields;
    for (auto &line : rows) {
        std::string t = replace_all(line, "|||", "");
        t = replace_all(t, "||", "");
        t = drop_nondigit_pipe_nondigit(t);
        t = drop_nondigit_pipe_nondigit(t);
        t = unphased_to_missing(t);
        for (auto &c : t)
            if (c == '|') c = '\t';
        for (auto &c : t)
            if (c == '.') c = '4';
        std::vector<std::string> f;
        size_t pos = 0;
        for (;;) {
            size_t e = t.find('\t', pos);
            if (e == std::string::npos) {
                f.push_back(t.substr(pos));
                break;
            }
            f.push_back(t.substr(pos, e - pos));
            pos = e + 1;
        }
        // del t[2:9]; del t[0]
        if (f.size() > 2) f.erase(f.begin() + 2, f.begin() + std::min<size_t>(9, f.size()));
        if (!f.empty()) f.erase(f.begin());
        fields.push_back(std::move(f));
    }
    fields.pop_back();  // del data[len(data)-1] (WeightedLD.py:365)
    if (fields.empty()) return fail(WLD_E_FORMAT, "%s: no variants left after dropping the last line", path);
    size_t width = fields[0].size();
    for (auto &f : fields)
        if (f.size() != width || width < 2)
            return fail(WLD_E_FORMAT, "%s: ragged VCF rows (numpy would build an object array)", path);
    const size_t L = fields.size(), N = width - 1;
    auto *ss = new wld_siteset;
    SiteSet &s = ss->s;
    s.n_sites = L;
    s.n_seqs = N;
    s.has_map = true;
    s.site_map.resize(L);
    s.buffer.resize(L * N);
    for (size_t i = 0; i < L; ++i) {
        long long v;
        if (!parse_int(fields[i][0], v)) {
            delete ss;
            return fail(WLD_E_FORMAT, "%s: bad POS '%s'", path, fields[i][0].c_str());
        }
        s.site_map[i] = (uint64_t)v;
        for (size_t h = 0; h < N; ++h) {
            if (!parse_int(fields[i][1 + h], v)) {
                delete ss;
                return fail(WLD_E_FORMAT, "%s: bad genotype '%s'", path, fields[i][1 + h].c_str());
            }
            uint8_t code = (uint8_t)(v & 0xFF);  // int64 -> uint8 wraps (numpy astype)
            if (code > WLD_SYM_UNKNOWN) code = WLD_SYM_UNKNOWN;
            // np.rot90: sequence q is haplotype column N-1-q
            s.buffer[i * N + (N - 1 - h)] = code;
        }
    }
    compute_histograms(s);
    *out = ss;
    return WLD_OK;
}

}  // extern "C"
