// Checks wld_tsv::fmt3 / fmt_u64 (weightedld_amd/csrc/tsv_format.hpp) against
// snprintf("%.3f") / ("%llu").  Modes:
//   tsv_format_check sample <n> <seed>   edge cases + n random bit patterns
//   tsv_format_check range <lo> <hi>     every bit pattern in [lo, hi)
// Prints "mismatches=<k> checked=<n>" and the first few mismatches.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "tsv_format.hpp"

static uint64_t checked = 0, bad = 0;

static void ref3(char *out, float v) {
    if (std::isnan(v)) { strcpy(out, "NaN"); return; }
    if (std::isinf(v)) { strcpy(out, v > 0 ? "inf" : "-inf"); return; }
    snprintf(out, 64, "%.3f", (double)v);
}

static void check_bits(uint32_t b) {
    float v;
    memcpy(&v, &b, 4);
    char a[80], r[80];
    int n = wld_tsv::fmt3(a, v);
    a[n] = 0;
    ref3(r, v);
    ++checked;
    if (strcmp(a, r)) {
        if (bad < 10) printf("bits=%08x got=%s want=%s\n", b, a, r);
        ++bad;
    }
}

static void check_u64(uint64_t v) {
    char a[32], r[32];
    int n = wld_tsv::fmt_u64(a, v);
    a[n] = 0;
    snprintf(r, sizeof r, "%" PRIu64, v);
    ++checked;
    if (strcmp(a, r)) {
        if (bad < 10) printf("u64=%" PRIu64 " got=%s\n", v, a);
        ++bad;
    }
}

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    std::string mode = argv[1];
    if (mode == "sample") {
        uint64_t n = strtoull(argv[2], 0, 10), s = strtoull(argv[3], 0, 10) | 1;
        const float edges[] = {0.0f, -0.0f, 1e-45f, -1e-45f, 0.0005f, -0.0005f, 0.0015f, 0.0625f, -0.0625f,
                               0.1875f, 0.3125f, 0.5f, 1.0f, -1.0f, 0.9995f, 2147483520.0f, 2147483648.0f,
                               -2147483648.0f, 3.4028235e38f, -3.4028235e38f, 1.17549435e-38f, 123.4565f};
        for (float e : edges) {
            uint32_t b;
            memcpy(&b, &e, 4);
            check_bits(b);
        }
        // every k/16 and k/2000 neighbourhood below 64 (exact ties and near-ties)
        for (int k = -1024; k <= 1024; ++k) {
            float t = k / 16.0f;
            uint32_t b;
            memcpy(&b, &t, 4);
            for (int d = -2; d <= 2; ++d) check_bits(b + d);
        }
        for (int k = -128000; k <= 128000; ++k) {
            float t = (float)(k / 2000.0);
            uint32_t b;
            memcpy(&b, &t, 4);
            for (int d = -1; d <= 1; ++d) check_bits(b + d);
        }
        check_bits(0x7fc00000u);
        check_bits(0xffc00001u);
        check_bits(0x7f800000u);
        check_bits(0xff800000u);
        for (uint64_t i = 0; i < n; ++i) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            check_bits((uint32_t)s);
            // values in the LdStats range [-1, 1] drawn uniformly in value
            float u = (float)((int64_t)(s >> 11) % 2000001 - 1000000) / 1000000.0f;
            uint32_t b;
            memcpy(&b, &u, 4);
            check_bits(b);
            check_u64(s >> (s & 63));
        }
        for (uint64_t v : {0ull, 9ull, 10ull, 4294967295ull, 18446744073709551615ull}) check_u64(v);
    } else if (mode == "range") {
        uint64_t lo = strtoull(argv[2], 0, 0), hi = strtoull(argv[3], 0, 0);
        for (uint64_t b = lo; b < hi; ++b) check_bits((uint32_t)b);
    } else {
        return 2;
    }
    printf("mismatches=%" PRIu64 " checked=%" PRIu64 "\n", bad, checked);
    return bad ? 1 : 0;
}
