// Host check of the epilogue's quotients by total_weight (pair_common.hpp
// ld_epilogue, WLD_EPI_DIVT): RN_f32(x * r) in f64 with r refined by two
// Newton steps from a coarse estimate (here the f32 reciprocal, ~2^-24; the
// device starts from v_rcp_f64) must equal the IEEE f32 quotient x / T for
// every pair tried.  Random significands over wide exponent ranges, x and T
// near each other, x / T near 1, subnormal quotients, integer-valued sums,
// powers of two, subnormal T.  Prints the mismatch count; exits 1 on any.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "pair_common.hpp"

static float bits(uint32_t b) {
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 20000000;
    std::mt19937_64 rng(12345);
    long bad = 0, tried = 0;
    auto check = [&](float x, float t) {
        if (!(t != 0.0f) || !std::isfinite(t) || !std::isfinite(x)) return;
        const double r = wld::recip_f64((double)t, wld::recip_seed_host(t));
        const float q = (float)((double)x * r), ref = x / t;
        ++tried;
        uint32_t a, b;
        std::memcpy(&a, &q, 4);
        std::memcpy(&b, &ref, 4);
        if (a != b) {
            if (bad < 10) printf("x %.9g t %.9g: %.9g vs %.9g\n", x, t, q, ref);
            ++bad;
        }
    };
    std::uniform_int_distribution<uint32_t> mant(0, (1u << 23) - 1), ex(1, 254), small(0, 60);
    for (long i = 0; i < n; ++i) {
        const uint32_t mt = mant(rng), mx = mant(rng);
        switch (i % 7) {
        case 0:  // anything
            check(bits(ex(rng) << 23 | mx), bits(ex(rng) << 23 | mt));
            break;
        case 1: {  // x <= T, close exponents (the epilogue's normalised quantities)
            const uint32_t e = 100 + small(rng);
            check(bits((e - small(rng) % 30) << 23 | mx), bits(e << 23 | mt));
            break;
        }
        case 2: {  // x / T near 1
            const uint32_t e = ex(rng);
            check(bits(e << 23 | mx), bits(e << 23 | (mx ^ (1u << small(rng) % 8))));
            break;
        }
        case 3:  // integer sums (unit weights)
            check((float)(rng() % 100000), (float)(1 + rng() % 100000));
            break;
        case 4:  // subnormal quotients
            check(bits((1 + small(rng)) << 23 | mx), bits((100 + small(rng)) << 23 | mt));
            break;
        case 6:  // subnormal T (quotients up to overflow)
            check(bits(ex(rng) % 160 << 23 | mx), bits(mt ? mt : 1u));
            break;
        default:  // powers of two and all-ones significands
            check(bits(ex(rng) << 23 | ((i & 8) ? 0x7FFFFFu : 0u)), bits(ex(rng) << 23 | ((i & 16) ? 0x7FFFFFu : mt)));
            break;
        }
    }
    printf("tried %ld mismatches %ld\n", tried, bad);
    return bad != 0;
}
