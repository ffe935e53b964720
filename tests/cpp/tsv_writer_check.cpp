// Writes synthetic pair rows with the CLI's pipelined write_pair_stats
// (weightedld_amd/csrc/cli.cpp, compiled in with its main renamed) and
// compares the file byte-for-byte with a serial snprintf writer.
//   tsv_writer_check <rows> <out_dir>
#define main weighted_ld_cli_main
#include "cli.cpp"
#undef main

#include <fstream>
#include <sstream>

static std::string slurp(const std::string &p) {
    std::ifstream f(p, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const uint64_t n = strtoull(argv[1], 0, 10);
    const std::string dir = argv[2];
    const bool realistic = argc > 3;  // LdStats-range values only (timing runs)
    std::vector<uint32_t> a(n), b(n);
    std::vector<float> d(n), dp(n), r2(n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        a[i] = (uint32_t)(i / 1000);
        b[i] = (uint32_t)(s >> 40);
        uint32_t bits = (uint32_t)s;
        memcpy(&d[i], &bits, 4);  // any bit pattern: NaN, inf, huge, subnormal
        dp[i] = (float)((int64_t)(s >> 20) % 2000001 - 1000000) / 1000000.0f;
        r2[i] = (float)(s >> 45) / (float)(1ull << 19) / 16.0f * 16.0f;
        if (realistic) d[i] = dp[i] * 0.25f;
    }
    wld_pairs p{};
    p.n = n;
    p.site_a = a.data();
    p.site_b = b.data();
    p.d = d.data();
    p.d_prime = dp.data();
    p.r2 = r2.data();
    const std::string got = dir + "/pipelined.tsv", want = dir + "/serial.tsv";
    const auto t0 = std::chrono::steady_clock::now();
    if (write_pair_stats(got, p) != WLD_OK) return 3;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    FILE *f = fopen(want.c_str(), "wb");
    fputs("site_a\tsite_b\td\td'\tr2\n", f);
    auto ref3 = [](float v) -> std::string {
        char t[80];
        if (std::isnan(v)) return "NaN";
        if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
        snprintf(t, sizeof t, "%.3f", (double)v);
        return t;
    };
    for (uint64_t i = 0; i < n; ++i)
        fprintf(f, "%u\t%u\t%s\t%s\t%s\n", a[i], b[i], ref3(d[i]).c_str(), ref3(dp[i]).c_str(), ref3(r2[i]).c_str());
    fclose(f);
    const bool same = slurp(got) == slurp(want);
    printf("rows=%llu identical=%d write_ms=%.1f\n", (unsigned long long)n, (int)same, ms);
    return same ? 0 : 1;
}
