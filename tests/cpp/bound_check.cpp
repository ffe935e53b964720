// Host harness for r2_bound_skip (pair_common.hpp), the pair kernels' skip
// test: reads records {T, A, B, AB, R (f64), thr (f64), nonneg (f64)} from
// argv[1], writes one byte per record (1 = skip) to argv[2].
#include <cstdio>
#include <vector>

#include "pair_common.hpp"

int main(int argc, char **argv) {
    if (argc != 3) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 3;
    std::vector<double> rec;
    double buf[7];
    while (fread(buf, sizeof(double), 7, f) == 7) rec.insert(rec.end(), buf, buf + 7);
    fclose(f);
    const size_t n = rec.size() / 7;
    std::vector<unsigned char> out(n);
    for (size_t i = 0; i < n; ++i) {
        const double *r = &rec[7 * i];
        out[i] = wld::r2_bound_skip(r[0], r[1], r[2], r[3], r[4], (float)r[5], r[6] != 0.0) ? 1 : 0;
    }
    FILE *g = fopen(argv[2], "wb");
    if (!g) return 4;
    fwrite(out.data(), 1, n, g);
    fclose(g);
    return 0;
}
