// Host harness for r2_bound_skip (pair_common.hpp), the pair kernels' skip
// test: reads records {T, A, B, AB, R (f64), thr (f64), nonneg (f64)} from
// argv[1], writes one byte per record (1 = skip) to argv[2].  With argv[3] =
// "f32": the screen's f32 form r2_screen_skip_f32 (inputs rounded to f32, R
// rounded up; nonneg ignored — the f32 form is for nonnegative weights only).
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "pair_common.hpp"

int main(int argc, char **argv) {
    if (argc != 3 && argc != 4) return 2;
    const bool f32 = argc == 4 && std::string(argv[3]) == "f32";
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
        if (f32) {
            float R = (float)r[4];
            if ((double)R < r[4]) R = std::nextafter(R, INFINITY);
            out[i] = wld::r2_screen_skip_f32((float)r[0], (float)r[1], (float)r[2], (float)r[3], R, (float)r[5]) ? 1 : 0;
        } else {
            out[i] = wld::r2_bound_skip(r[0], r[1], r[2], r[3], r[4], (float)r[5], r[6] != 0.0) ? 1 : 0;
        }
    }
    FILE *g = fopen(argv[2], "wb");
    if (!g) return 4;
    fwrite(out.data(), 1, n, g);
    fclose(g);
    return 0;
}
