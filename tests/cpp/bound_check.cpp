// Host harness for r2_bound_skip (pair_common.hpp), the pair kernels' skip
// test: reads records {T, A, B, AB, R (f64), thr (f64), nonneg (f64)} from
// argv[1], writes one byte per record (1 = skip) to argv[2].  With argv[3] =
// "f32": the screen's f32 form r2_screen_skip_f32 (inputs rounded to f32, R
// rounded up; nonneg ignored — the f32 form is for nonnegative weights only).
// With argv[3] = "f32g": the screen kernel's split form (screen_consts from a
// launch-wide bound Tg >= T, passed in the nonneg field, then r2_screen_terms;
// skip iff both terms are <= 0).  "f32xy": the same from the accumulator form
// (X0 = (T + B) / 2, Y0 = (T - B) / 2, X1 = (A + AB) / 2, Y1 = (A - AB) / 2;
// r2_screen_terms_xy).  "f32fg": the fp6 screen's form (F0 = T - B/2, G0 =
// T - 3B/4, F1 = A - AB/2, G1 = A - 3AB/4 of the doubled record sums; R put on
// the accumulators' grid, here 1/2, as the kernel does; r2_screen_terms_fg,
// skip iff t1 <= 0 and every marginal >= mloc).  "f32xy2": r2_screen_terms_xy2
// on the X/Y accumulators, R on the same grid, the same skip rule.
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "pair_common.hpp"

int main(int argc, char **argv) {
    if (argc != 3 && argc != 4) return 2;
    const bool f32 = argc == 4 && std::string(argv[3]) == "f32";
    const bool f32xy = argc == 4 && std::string(argv[3]) == "f32xy";
    const bool f32fg = argc == 4 && std::string(argv[3]) == "f32fg";
    const bool f32xy2 = argc == 4 && std::string(argv[3]) == "f32xy2";
    const bool f32g = f32xy || f32fg || f32xy2 || (argc == 4 && std::string(argv[3]) == "f32g");
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
        if (f32g) {
            float R = (float)r[4], Tg = (float)r[6];
            if ((double)R < r[4]) R = std::nextafter(R, INFINITY);
            if (f32fg || f32xy2) R = (float)(std::ceil(r[4] * 2.0) / 2.0);
            if ((double)Tg < r[6]) Tg = std::nextafter(Tg, INFINITY);
            float E, mloc, t2;
            wld::screen_consts(Tg, R, E, mloc);
            const float thr_c = (float)r[5] * (1.0f - 0x1p-7f);
            if (f32xy2) {
                float mlo;
                const float t1 = wld::r2_screen_terms_xy2((float)((r[0] + r[2]) / 2), (float)((r[0] - r[2]) / 2),
                                                          (float)((r[1] + r[3]) / 2), (float)((r[1] - r[3]) / 2), R,
                                                          thr_c, E, mlo);
                out[i] = t1 <= 0.0f && mlo >= mloc ? 1 : 0;
                continue;
            }
            if (f32fg) {
                float mlo;
                const float t1 = wld::r2_screen_terms_fg((float)(r[0] - r[2] / 2), (float)(r[0] - 0.75 * r[2]),
                                                         (float)(r[1] - r[3] / 2), (float)(r[1] - 0.75 * r[3]), R,
                                                         thr_c, E, mlo);
                out[i] = t1 <= 0.0f && mlo >= mloc ? 1 : 0;
                continue;
            }
            const float t1 =
                f32xy ? wld::r2_screen_terms_xy((float)((r[0] + r[2]) / 2), (float)((r[0] - r[2]) / 2),
                                                (float)((r[1] + r[3]) / 2), (float)((r[1] - r[3]) / 2), R, thr_c, E,
                                                mloc, t2)
                      : wld::r2_screen_terms((float)r[0], (float)r[1], (float)r[2], (float)r[3], R, thr_c, E, mloc, t2);
            out[i] = t1 <= 0.0f && t2 <= 0.0f ? 1 : 0;
        } else if (f32) {
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
