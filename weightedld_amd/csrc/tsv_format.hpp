// TSV field formatting for the CLI writer (main.rs:76,82-119): site indices as
// `{}` and f32 statistics as Rust `{:.3}`.
//
// Rust formats `{:.3}` from the exact binary value with round-half-to-even on
// ties (flt2dec format_exact), which is what glibc's "%.3f" of the widened
// double does too; NaN and the infinities use Rust's spellings ("NaN", "inf",
// "-inf").  fmt3 computes round(|v|*1000) in integer arithmetic for
// |v| < 2^31 (every value an LdStats row holds in practice) and falls back to
// snprintf above that.  tests/test_tsv_format.py checks it against snprintf.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

namespace wld_tsv {

// Decimal digits of v (no sign), returns the length.
inline int fmt_u64(char *out, uint64_t v) {
    char tmp[20];
    int n = 0;
    do {
        tmp[n++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    for (int i = 0; i < n; ++i) out[i] = tmp[n - 1 - i];
    return n;
}

inline int fmt3(char *out, float v) {
    uint32_t bits;
    memcpy(&bits, &v, 4);
    const bool neg = bits >> 31;
    const uint32_t ex = (bits >> 23) & 0xFF;
    uint32_t man = bits & 0x7FFFFF;
    if (ex == 0xFF) {
        if (man) {
            memcpy(out, "NaN", 3);
            return 3;
        }
        if (neg) {
            memcpy(out, "-inf", 4);
            return 4;
        }
        memcpy(out, "inf", 3);
        return 3;
    }
    // |v| = man * 2^e2
    int e2;
    if (ex == 0) {
        e2 = -149;
    } else {
        man |= 0x800000;
        e2 = (int)ex - 150;
    }
    if (e2 > 7)  // |v| >= 2^31: rare, exact libc path
        return snprintf(out, 64, "%.3f", (double)v);
    const uint64_t x = (uint64_t)man * 1000u;  // < 2^34
    uint64_t q;
    if (e2 >= 0) {
        q = x << e2;
    } else if (e2 > -64) {
        const int s = -e2;
        q = x >> s;
        const uint64_t rem = x & ((uint64_t(1) << s) - 1), half = uint64_t(1) << (s - 1);
        if (rem > half || (rem == half && (q & 1))) ++q;
    } else {
        q = 0;  // x < 2^34 < half
    }
    int n = 0;
    if (neg) out[n++] = '-';
    n += fmt_u64(out + n, q / 1000);
    const uint32_t f = (uint32_t)(q % 1000);
    out[n] = '.';
    out[n + 1] = (char)('0' + f / 100);
    out[n + 2] = (char)('0' + (f / 10) % 10);
    out[n + 3] = (char)('0' + f % 10);
    return n + 4;
}

}  // namespace wld_tsv
