// Device helpers shared by the pair kernels: the LdStats epilogue and the
// tile compaction that feeds the reference-order gather (order.hip).
#pragma once

#include "kernels.hpp"

namespace wld {

// lib.rs:482-520, operation for operation in f32 (the library is built with
// -ffp-contract=off, divisions are IEEE-rounded, fminf/fmaxf ignore NaN like
// Rust's f32::min/max).  Inputs are the four masked weight sums of
// lib.rs:423-480: total_weight, PA (a major), PB (b major), ld_obs[3] (both).
__device__ __forceinline__ void ld_epilogue(float total_weight, float PA, float PB, float ld3, float &d_out,
                                            float &dp_out, float &r2_out) {
    float ld_obs0, ld_obs1, ld_obs2, ld_obs3 = ld3;
    float Pa = total_weight - PA;
    float Pb = total_weight - PB;
    ld_obs2 = PA - ld_obs3;
    ld_obs1 = PB - ld_obs3;
    ld_obs0 = Pa - ld_obs1;
    PA = PA / total_weight;
    PB = PB / total_weight;
    Pa = Pa / total_weight;
    Pb = Pb / total_weight;
    ld_obs0 = ld_obs0 / total_weight;
    ld_obs1 = ld_obs1 / total_weight;
    ld_obs2 = ld_obs2 / total_weight;
    ld_obs3 = ld_obs3 / total_weight;
    const float PAB = PA * PB;
    const float PAb = PA * Pb;
    const float PaB = Pa * PB;
    const float Pab = Pa * Pb;
    const float d = ((PAB - ld_obs3) + (Pab - ld_obs0) + (ld_obs2 - PAb) + (ld_obs1 - PaB)) / 4.0f;
    float den;
    if (d < 0.0f) {
        den = fmaxf(-ld_obs0, -ld_obs3);
        if (den == 0.0f) den = fminf(-ld_obs0, -ld_obs3);
    } else {
        den = fminf(ld_obs1, ld_obs2);
        if (den == 0.0f) den = fmaxf(ld_obs1, ld_obs2);
    }
    d_out = d;
    dp_out = d / den;
    r2_out = d * d / (PA * Pa * PB * Pb);
}

__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    return v;
}

}  // namespace wld
