// f32 pair kernel: the exact-f32 path, the fallback for weights the integer
// MFMA kernel's fixed-point planes cannot hold exactly, and the reference-order
// path (WLD_OPT_REF_SUMS).  For finite weights the products and sums run on
// f32-input MFMA (MF below); the VALU loop described next is the SAFE
// (non-finite weights) path and the WLD_VALU_PLAIN=1 variant.
//
// Replaces the inner loop of single_weighted_ld_pair (lib.rs:416-480) for a
// 64x64 tile of site pairs per 256-thread workgroup.  Each thread owns a 4x4
// block of pairs (a = a0 + ty + 16i, b = b0 + tx + 16j) and keeps the four
// weighted masked sums of lib.rs:441-444 per pair in registers:
//     T   += w  where a in {maj,min} and b in {maj,min}
//     SA  += w  where additionally a == maj
//     SB  += w  where additionally b == maj
//     SAB += w  where a == maj and b == maj
// as fmaf(u, f, acc) with u = w or 0 (a side) and f = 1.0 or 0.0 (b side):
// w*1 and w*0 are exact, so each sum is an f32 sum over sequences in order
// (the same terms in the same order for all four sums, so SA == T still
// implies SAB == SB exactly and degenerate pairs stay NaN as in the
// reference).  (The SAFE variant uses selects, for non-finite weights where
// 0*inf would differ from the reference's select.)  Codes of both 64-site
// panels and the weights are staged through LDS 64 sequences at a time.
//
// Summation blocks.  acc holds the current block of 64-sequence stages, tot
// the running total:
//   * default: blocks of `flush` stages (about sqrt(N) sequences), tot += acc
//     after each (~2 sqrt(N) 2^-24 relative error, below the reference's own);
//   * REF (WLD_OPT_REF_SUMS): the reference's own f32 order, lib.rs:416-480.
//     The sequences are permuted at load (ref_layout_kernel) into the lane
//     classes of the 8-lane loop: block j (j = 0..7) holds sequences j, j+8,
//     j+16, ... < 8 floor(N/8) in order, zero padded to `cs` stages, then one
//     stage with the scalar tail (sequences 8 floor(N/8) .. N-1).  Block j's
//     chain from 0 is lane j's f32x8 sum (lib.rs:441-444: each add rounds
//     once, adding a masked-out 0 is exact); tot += acc after block j is the
//     ordered horizontal sum ((((0 + l0) + l1) + ...) + l7) that packed_simd's
//     f32x8::sum() computes on x86 (lib.rs:447-452); the <= 7 tail sequences
//     are then added onto tot one by one on the VALU, as the scalar loop adds
//     onto the horizontal sums (lib.rs:461-480).  With the epilogue op for
//     op, the rows are bit-identical to lib.rs.  Inside a class each group of
//     16 positions is stored transposed (position 4g + j holds element 4j + g
//     of the group): the MFMA's lane group g takes element 4j + g at step j,
//     so one dword read gives a lane its codes (one 16-byte read its weights)
//     for four steps.
// With LOOP the workgroup strides over a tile list whose length is known only
// on the device (the candidate tiles of the i8 screen, pair_mfma.hip), and
// the last workgroup runs the run's chunk scan (scan_tail).
#include "pair_common.hpp"

namespace wld {

namespace {
constexpr int kStride = 68;  // LDS row stride in bytes (17 dwords: conflict-free b reads)
}

typedef float v4f __attribute__((ext_vector_type(4)));

// MF = true: the products and f32 sums of the non-SAFE path on the matrix
// cores, v_mfma_f32_16x16x4_f32 (f32 inputs, exact products, an f32 fma chain
// over k, bitwise equal to a sequential fmaf loop: MI355X_MICROARCH.md, Matrix
// cores).  Wave w owns a rows 16w..16w+15 against the tile's 64 b columns in
// four 16x16 blocks; lane l = 16g + r carries a row r (A) / b column r (B) at
// sequence kk + g, and holds the sums of pairs (a = 16w + 4g + e, b = 16n + r)
// — the same thread -> (4 a rows, 4 b columns) shape as the VALU mapping (a =
// ty + 16i), so the epilogue and compaction only change how a row slot maps
// to a.  The VALU's code extraction then overlaps the matrix pipe instead of
// competing with the FMAs for VALU issue.
#ifndef WLD_VALU_MF_WG
#define WLD_VALU_MF_WG 2  // MF: 164 VGPRs would fit 3 per CU; measured equal
#endif
#ifndef WLD_VALU_REF_WG
#define WLD_VALU_REF_WG 3  // MF + REF: three workgroups per CU (<= 168 VGPRs; 2 leave 208)
#endif
template <bool DENSE, bool SAFE, bool MF, bool REF, bool LOOP>
__global__ __launch_bounds__(256, MF ? (REF ? WLD_VALU_REF_WG : WLD_VALU_MF_WG) : 2) void pair_valu_kernel(
    const uint8_t *__restrict__ codes, const float *__restrict__ w, const uint8_t *__restrict__ site_ok,
    const uint32_t *__restrict__ tiles, uint32_t n_tiles, const unsigned *tile_count,
    const uint32_t *__restrict__ tile_bits, unsigned *tile_work, const unsigned *tile_buckets, uint32_t bucket_cap,
    uint32_t L, uint32_t NP, uint32_t flush,
    uint32_t ref_cs, uint32_t ref_tail_n, uint32_t n_chunk_rows, float thr, OrderArgs o, DenseArgs dn, ScanArgs sa) {
    constexpr int NS = 4;  // 16x16 slots per wave: a whole 64x64 tile per workgroup
    __shared__ __attribute__((aligned(16))) uint8_t sA[kTile * kStride];
    __shared__ __attribute__((aligned(16))) uint8_t sB[kTile * kStride];
    __shared__ __attribute__((aligned(16))) float sW[64];
    __shared__ unsigned long long sBits[kTile];  // compaction: passing b per a row
    __shared__ uint32_t sRowBase[kTile];

    // bits: the 16x16 sub-blocks whose pairs are computed (bit 4 (a / 16) +
    // b / 16); the others' pairs provably fail (the screen's bound).  owned:
    // the tile's 16-row blocks whose segment counts this work item writes (a
    // tile split over several items gives each its own row blocks)
    auto compute_tile = [&](uint32_t tile, uint32_t tid, uint32_t bits, uint32_t owned) {
        const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;
        const uint32_t a0 = ta * kTile, b0 = tb * kTile;
        const uint32_t tx = tid & 15, ty = tid >> 4;

        float acc[4][4][4], tot[4][NS][4];
        v4f accM[NS][4];  // MF: [slot j][sum q], element e = a row slot
        // MF + REF: the computed sub-blocks dealt over the waves.  In
        // column-major order (k = 4 n + i: a rows 16 i.., b columns 16 n..)
        // the u-th computed one goes to wave u % 4, slot u / 4: the stage
        // barriers pace a tile by its busiest wave, and a diagonal tile's 10
        // sub-blocks then take 3 slots on it instead of 4; all 16 give wave w
        // the a rows 16 w.. against b block j in slot j.
        uint32_t ui[NS], un[NS];
        bool us[NS];
#pragma unroll
        for (int j = 0; j < NS; ++j) ui[j] = 0, un[j] = j, us[j] = true;
        if constexpr (MF && REF) {
            const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
            uint32_t cm = 0;
            for (uint32_t k = 0; k < 16; ++k) cm |= ((bits >> (4 * (k & 3) + (k >> 2))) & 1u) << k;
            cm = __builtin_amdgcn_readfirstlane(cm);
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                uint32_t m = cm;
                for (uint32_t t = 0; t < 4 * (uint32_t)j + wave; ++t) m &= m - 1u;  // drop the first 4j + w
                const uint32_t k = m ? (uint32_t)__builtin_ctz(m) : 0u;
                us[j] = m != 0;
                ui[j] = k & 3u;
                un[j] = k >> 2;
            }
        }
        // the tile's a row / b column of this thread's pair (row slot i, slot j)
        auto pa = [&](int i, int j) -> uint32_t {
            if constexpr (MF && REF) return 16 * ui[j] + 4 * (ty & 3) + i;
            else return MF ? 4 * ty + i : ty + 16 * i;
        };
        auto pb = [&](int i, int j) -> uint32_t {
            if constexpr (MF && REF) return 16 * un[j] + tx;
            else return tx + 16 * j;
        };
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NS; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) tot[i][j][q] = 0.0f;

        const uint32_t lr = tid >> 2, part = tid & 3;  // loader: site row, 16-byte part
        const uint8_t *gA = codes + (size_t)(a0 + lr) * NP + part * 16;
        const uint8_t *gB = codes + (size_t)(b0 + lr) * NP + part * 16;

        // one 64-sequence stage of both panels' codes and the weights: fetch
        // (global loads into registers, issued a stage ahead so that their
        // latency overlaps the previous stage's MFMAs), then store (into LDS).
        // PF: the fetch a stage ahead; a whole tile per workgroup in lib.rs's
        // order has no registers to spare for it (it would spill), and fetches
        // each stage just before storing it
        constexpr bool PF = !REF;
        uint4 va, vb;
        float wv;
        auto fetch_stage = [&](uint32_t k0) {
            va = *reinterpret_cast<const uint4 *>(gA + k0);
            vb = *reinterpret_cast<const uint4 *>(gB + k0);
            wv = tid < 64 ? w[k0 + tid] : 0.0f;
        };
        auto store_stage = [&]() {
            __syncthreads();
            uint32_t *pa = reinterpret_cast<uint32_t *>(sA + lr * kStride + part * 16);
            uint32_t *pb = reinterpret_cast<uint32_t *>(sB + lr * kStride + part * 16);
            pa[0] = va.x, pa[1] = va.y, pa[2] = va.z, pa[3] = va.w;
            pb[0] = vb.x, pb[1] = vb.y, pb[2] = vb.z, pb[3] = vb.w;
            if (tid < 64) sW[tid] = wv;
            __syncthreads();
        };
        // the staged 64 sequences into acc (VALU) / accM (MF), in sequence order
        auto compute_stage = [&]() {
            if constexpr (MF && REF) {
                // transposed 16-position groups: lane (r, g) reads the dword of
                // its row at 16 grp + 4 g = elements 16 grp + 4 e + g, e = 0..3;
                // slot j (a rows 16 ui[j].., b block un[j]) runs its 16 MFMAs of
                // the group when the wave holds it (us[j], wave-uniform)
                const uint32_t lane = tid & 63, r = lane & 15, g = lane >> 4;
#pragma unroll
                for (int grp = 0; grp < 4; ++grp) {
                    const float4 w4 = *reinterpret_cast<const float4 *>(sW + 16 * grp + 4 * g);
                    const float we[4] = {w4.x, w4.y, w4.z, w4.w};
                    float u[4], v[4];
#pragma unroll
                    for (int j = 0; j < NS; ++j) {
                        if (!us[j]) continue;  // (slots fill in order: us[j] implies us[j - 1])
                        if (j == 0 || ui[j] != ui[j - 1]) {  // a rows of a new row block (all 16: slot 0 only)
                            const uint32_t a4 =
                                *reinterpret_cast<const uint32_t *>(sA + (16 * ui[j] + r) * kStride + 4 * g + 16 * grp);
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const uint32_t ca = a4 >> (8 * e);
                                u[e] = (ca & kCodeIn) ? we[e] : 0.0f;
                                v[e] = (ca & kCodeMaj) ? we[e] : 0.0f;
                            }
                        }
                        const uint32_t b4 =
                            *reinterpret_cast<const uint32_t *>(sB + (16 * un[j] + r) * kStride + 4 * g + 16 * grp);
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float fi = (float)((b4 >> (8 * e)) & 1u), fm = (float)((b4 >> (8 * e + 1)) & 1u);
                            accM[j][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[e], fi, accM[j][0], 0, 0, 0);
                            accM[j][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[e], fi, accM[j][1], 0, 0, 0);
                            accM[j][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[e], fm, accM[j][2], 0, 0, 0);
                            accM[j][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[e], fm, accM[j][3], 0, 0, 0);
                        }
                    }
                }
            } else if constexpr (MF) {
                const uint32_t lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
                const uint8_t *rowA = sA + (16 * wave + r) * kStride + g;
                const uint8_t *rowB = sB + r * kStride + g;
#pragma unroll 4
                for (int kk = 0; kk < 64; kk += 4) {
                    const float we = sW[kk + g];
                    const uint32_t ca = rowA[kk];
                    const float u = (ca & kCodeIn) ? we : 0.0f;
                    const float v = (ca & kCodeMaj) ? we : 0.0f;
#pragma unroll
                    for (int n = 0; n < 4; ++n) {
                        const uint32_t cb = rowB[16 * n * kStride + kk];
                        const float fi = (float)(cb & 1u), fm = (float)(cb >> 1);
                        accM[n][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, fi, accM[n][0], 0, 0, 0);
                        accM[n][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, fi, accM[n][1], 0, 0, 0);
                        accM[n][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, fm, accM[n][2], 0, 0, 0);
                        accM[n][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, fm, accM[n][3], 0, 0, 0);
                    }
                }
            } else {
#pragma unroll 2
                for (int kk = 0; kk < 64; kk += 4) {
                    uint32_t A[4], B[4];
                    float wk[4];
                    if constexpr (REF) {
                        // elements kk + e (e = 0..3) of the transposed group
                        // sit at 16 (kk / 16) + 4 e + (kk % 16) / 4
                        const int p0 = 16 * (kk / 16) + (kk % 16) / 4;
                        auto gather = [&](const uint8_t *row) {
                            return (uint32_t)row[p0] | (uint32_t)row[p0 + 4] << 8 | (uint32_t)row[p0 + 8] << 16 |
                                   (uint32_t)row[p0 + 12] << 24;
                        };
#pragma unroll
                        for (int i = 0; i < 4; ++i) A[i] = gather(sA + (ty + 16 * i) * kStride);
#pragma unroll
                        for (int j = 0; j < 4; ++j) B[j] = gather(sB + (tx + 16 * j) * kStride);
#pragma unroll
                        for (int e = 0; e < 4; ++e) wk[e] = sW[p0 + 4 * e];
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            A[i] = *reinterpret_cast<const uint32_t *>(sA + (ty + 16 * i) * kStride + kk);
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            B[j] = *reinterpret_cast<const uint32_t *>(sB + (tx + 16 * j) * kStride + kk);
                        const float4 w4 = *reinterpret_cast<const float4 *>(sW + kk);
                        wk[0] = w4.x; wk[1] = w4.y; wk[2] = w4.z; wk[3] = w4.w;
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float we = wk[e];
                        float u[4], v[4];
                        uint32_t ca[4], cb[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            ca[i] = (A[i] >> (8 * e)) & 3u;
                            u[i] = (ca[i] & kCodeIn) ? we : 0.0f;
                            v[i] = (ca[i] & kCodeMaj) ? we : 0.0f;
                        }
#pragma unroll
                        for (int j = 0; j < 4; ++j) cb[j] = (B[j] >> (8 * e)) & 3u;
                        if constexpr (!SAFE) {
                            float fi[4], fm[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                fi[j] = (float)(cb[j] & 1u);
                                fm[j] = (float)(cb[j] >> 1);
                            }
#pragma unroll
                            for (int i = 0; i < 4; ++i)
#pragma unroll
                                for (int j = 0; j < 4; ++j) {
                                    acc[i][j][0] = __builtin_fmaf(u[i], fi[j], acc[i][j][0]);
                                    acc[i][j][1] = __builtin_fmaf(v[i], fi[j], acc[i][j][1]);
                                    acc[i][j][2] = __builtin_fmaf(u[i], fm[j], acc[i][j][2]);
                                    acc[i][j][3] = __builtin_fmaf(v[i], fm[j], acc[i][j][3]);
                                }
                        } else {
#pragma unroll
                            for (int i = 0; i < 4; ++i)
#pragma unroll
                                for (int j = 0; j < 4; ++j) {
                                    const bool bi = cb[j] & 1u, bm = cb[j] & 2u;
                                    acc[i][j][0] += bi ? u[i] : 0.0f;
                                    acc[i][j][1] += bi ? v[i] : 0.0f;
                                    acc[i][j][2] += bm ? u[i] : 0.0f;
                                    acc[i][j][3] += bm ? v[i] : 0.0f;
                                }
                        }
                    }
                }
            }
        };
        // block start: acc = 0; block end: tot += acc
        auto acc_zero = [&]() {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < NS; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if constexpr (MF) accM[j][q][i] = 0.0f;
                        else acc[i][j][q] = 0.0f;
                    }
        };
        auto acc_fold = [&]() {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < NS; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) tot[i][j][q] += MF ? accM[j][q][i] : acc[i][j][q];
        };

        if constexpr (REF) {
            // the eight lane classes, each a chain from 0 folded into the
            // ordered horizontal sum; then the tail stage on that sum.  The
            // stages are consecutive (class c's are [c cls, (c + 1) cls), the
            // tail's 8 cls), so each stage's fetch is issued before the
            // previous stage's compute.
            const uint32_t cls = 64 * ref_cs;
            if (PF && (ref_cs || ref_tail_n)) fetch_stage(0);
            for (uint32_t c = 0; c < (ref_cs ? 8u : 0u); ++c) {
                acc_zero();
                for (uint32_t k0 = c * cls; k0 < (c + 1) * cls; k0 += 64) {
                    if (!PF) fetch_stage(k0);
                    store_stage();
                    if (PF && (k0 + 64 < 8 * cls || ref_tail_n)) fetch_stage(k0 + 64);
                    compute_stage();
                }
                acc_fold();
            }
            if (ref_tail_n) {
                // the scalar tail (lib.rs:461-480): its <= 7 sequences added
                // onto the horizontal sums one by one, in order, on the VALU
                // (fmaf(u, f, tot) = tot + u f rounded once: u f is exact)
                if (!PF) fetch_stage(8 * cls);
                store_stage();
                for (uint32_t t = 0; t < ref_tail_n; ++t) {
                    const float we = sW[t];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < NS; ++j) {
                            const uint32_t ca = sA[pa(i, j) * kStride + t], cb = sB[pb(i, j) * kStride + t];
                            const float u = (ca & kCodeIn) ? we : 0.0f;
                            const float v = (ca & kCodeMaj) ? we : 0.0f;
                            if constexpr (!SAFE) {
                                const float fi = (float)(cb & 1u), fm = (float)(cb >> 1);
                                tot[i][j][0] = __builtin_fmaf(u, fi, tot[i][j][0]);
                                tot[i][j][1] = __builtin_fmaf(v, fi, tot[i][j][1]);
                                tot[i][j][2] = __builtin_fmaf(u, fm, tot[i][j][2]);
                                tot[i][j][3] = __builtin_fmaf(v, fm, tot[i][j][3]);
                            } else {
                                const bool bi = cb & 1u, bm = cb & 2u;
                                tot[i][j][0] += bi ? u : 0.0f;
                                tot[i][j][1] += bi ? v : 0.0f;
                                tot[i][j][2] += bm ? u : 0.0f;
                                tot[i][j][3] += bm ? v : 0.0f;
                            }
                        }
                }
            }
        } else {
            // blocks of `flush` stages
            fetch_stage(0);
            for (uint32_t k0 = 0; k0 < NP; k0 += 64 * flush) {
                acc_zero();
                for (uint32_t k1 = k0; k1 < min(NP, k0 + 64 * flush); k1 += 64) {
                    store_stage();
                    if (k1 + 64 < NP) fetch_stage(k1 + 64);
                    compute_stage();
                }
                acc_fold();
            }
        }

        // ---- epilogue ------------------------------------------------------
        uint32_t passmask[4] = {0, 0, 0, 0};  // bit j per row slot i
        float res[4][NS][3];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                const uint32_t al = pa(i, j), bl = pb(i, j), a = a0 + al, b = b0 + bl;
                float d, dp, r2;
                ld_epilogue(tot[i][j][0], tot[i][j][1], tot[i][j][2], tot[i][j][3], d, dp, r2);
                res[i][j][0] = d;
                res[i][j][1] = dp;
                res[i][j][2] = r2;
                // (every load issued, no short-circuit: a, b < LP; the compiler
                // batches them instead of one round trip per pair)
                const bool valid = (a < b) & (b < L) & ((site_ok[a] & site_ok[b]) != 0);
                if constexpr (DENSE) {
                    if (a < b && b < L) {
                        const size_t k = (size_t)a * L + b;
                        dn.d[k] = d;
                        dn.dp[k] = dp;
                        dn.r2[k] = r2;
                        dn.valid[k] = valid ? 1 : 0;
                    }
                } else {
                    // lib.rs:660 strict '>' (a skipped sub-block's pairs provably fail;
                    // an empty slot's pairs alias slot 0's sub-block)
                    if (valid && r2 > thr && us[j] && ((bits >> (4 * (al >> 4) + (bl >> 4))) & 1u))
                        passmask[i] |= 1u << j;
                }
            }
        }
        if constexpr (DENSE) return;

        // ---- compaction: a 64x64 pass-bit matrix in LDS, rows in b order ----
        // (a tile with no passing pair writes only its 64 zero counts)
        const bool own_row = tid < kTile && ((owned >> (tid >> 4)) & 1u);  // (row tid: its 16-row block)
        const uint32_t quarters = (uint32_t)__popc(owned);
        if (!__syncthreads_or((passmask[0] | passmask[1] | passmask[2] | passmask[3]) != 0)) {
            if (own_row) o.seg_cnt[(size_t)(a0 + tid) * o.T + tb] = 0;
            if (tid == 0) tile_done(o, ta, tb, n_chunk_rows, quarters);
            return;
        }
        if (tid < kTile) sBits[tid] = 0ull;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NS; ++j)
                if (passmask[i] & (1u << j)) atomicOr(&sBits[pa(i, j)], 1ull << pb(i, j));
        __syncthreads();
        if (tid < kTile) {
            const uint32_t r = tid;
            const uint32_t cnt = __popcll(sBits[r]);
            const uint32_t incl = wave_inclusive_scan(cnt);
            const uint32_t excl = incl - cnt;
            const uint32_t total = __shfl(incl, 63, 64);
            unsigned long long base = 0;
            if (r == 63 && total) base = atomicAdd(o.cursor, (unsigned long long)total);
            base = __shfl(base, 63, 64);
            sRowBase[r] = (uint32_t)base + excl;
            const uint32_t a = a0 + r;
            if (own_row) {  // (a row outside the item's blocks has no pass: cnt 0)
                o.seg_cnt[(size_t)a * o.T + tb] = (uint8_t)cnt;
                o.seg_off[(size_t)a * o.T + tb] = (uint32_t)base + excl;
            }
            if (r == 63 && total)
                atomicAdd(&o.chunk_total[chunk_linear(n_chunk_rows, ta / kTilesPerChunk, tb / kTilesPerChunk)], total);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (!passmask[i]) continue;
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                if (!(passmask[i] & (1u << j))) continue;
                const uint32_t al = pa(i, j), bl = pb(i, j);
                const uint64_t pos = (uint64_t)sRowBase[al] + __popcll(sBits[al] & ((1ull << bl) - 1ull));
                if (pos < o.st_capacity) {
                    o.st_a[pos] = a0 + al;
                    o.st_b[pos] = b0 + bl;
                    o.st_d[pos] = res[i][j][0];
                    o.st_dp[pos] = res[i][j][1];
                    o.st_r2[pos] = res[i][j][2];
                }
            }
        }
        if (tid == 0) tile_done(o, ta, tb, n_chunk_rows, quarters);
    };

    if constexpr (!LOOP) {
        const uint32_t tile = tiles[blockIdx.x];
        if (tile != kNoTile)  // kNoTile: padding of an XCD-ordered list
            compute_tile(tile, threadIdx.x, 0xFFFFu, 0xFu);
    } else {
        // (the list entries come from the screen's atomics: each is checked —
        // bucket slot, then the tile — before anything is read through it)
        // the first tile by workgroup id, the next ones from a work counter
        // (tile_work, zeroed by the screen): the workgroups that finish first
        // take the list's tail, not fixed ones (tiles differ in their computed
        // sub-blocks)
        __shared__ uint32_t s_next, s_pre[17];
        const uint32_t nt = (*tile_count & kAbandonBit) ? 0u : *tile_count;
        // first items: the list is heaviest first and the dispatcher deals
        // workgroups i, i + m, i + 2m, ... (m = grid / R, R resident per CU)
        // to one CU, so that CU would start R of the heaviest items at once
        // (one wave of each on every SIMD): deal the rounds in snake order
        // instead (j, 2m - 1 - j, 2m + j, ...), heavy next to light (a
        // permutation of [0, grid))
        uint32_t first = blockIdx.x;
        if (tile_buckets) {
            constexpr uint32_t R = WLD_VALU_REF_WG;
            const uint32_t m = gridDim.x / R, k = m ? blockIdx.x / m : R, j = blockIdx.x - (k < R ? k * m : 0u);
            if (k < R) first = (k & 1) ? (k + 1) * m - 1 - j : k * m + j;
        }
        if (tile_buckets && first < nt) cand_prefix(tile_buckets, s_pre);  // (a workgroup without a tile skips it)
        for (uint32_t bi = first; bi < nt;) {
            const uint32_t e = tile_buckets ? cand_entry_checked(o, s_pre, bucket_cap, bi) : bi < n_tiles ? bi : ~0u;
            const uint32_t tile = e != ~0u ? tiles[e] : kNoTile;
            // (a refused entry reads nothing through e: the guard has reported it)
            const uint32_t bits = tile_bits && e != ~0u ? tile_bits[e] : 0xFFFFu;
            if (tile_in_range(tile, L))
                compute_tile(tile, threadIdx.x, bits, 0xFu);  // (a whole-tile entry writes all 64 rows' segments)
            else if (e != ~0u && threadIdx.x == 0)
                report_guard(o, kGuardTile);
            if (threadIdx.x == 0) s_next = gridDim.x + atomicAdd(tile_work, 1u);
            __syncthreads();  // (also: the next tile's staging and compaction reuse the LDS)
            bi = s_next;
            __syncthreads();
        }
        scan_tail(sa, nt, false, first);
    }
}

// The reference-order layout (REF): sequence seq -> position p of the lane-
// class order.  Block j < 8 (cls positions each, cls = 0 when N < 8) holds
// seq = 8t + j at p = j cls + t' (t < floor(N/8)), t' = t with each group of
// 16 transposed (t = 16q + 4j + g at t' = 16q + 4g + j); the tail seq = 8
// floor(N/8) + t at p = 8 cls + t; every other position is padding (code 0,
// weight 0).  One thread per (site, position).
__global__ __launch_bounds__(256) void ref_layout_kernel(const uint8_t *__restrict__ codes, const float *__restrict__ w,
                                                         uint32_t LP, uint32_t NP, uint32_t N, uint32_t NPr,
                                                         uint32_t cls, uint8_t *__restrict__ rcodes,
                                                         float *__restrict__ rw) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)LP * NPr) return;
    const uint32_t s = (uint32_t)(idx / NPr), p = (uint32_t)(idx % NPr);
    const uint32_t n8 = N / 8;
    uint32_t seq = 0xFFFFFFFFu;
    if (p < 8 * cls) {
        const uint32_t blk = p / cls, tp = p % cls;
        const uint32_t t = (tp & ~15u) | (tp & 3u) << 2 | (tp >> 2 & 3u);  // transposed 16-groups
        if (t < n8) seq = 8 * t + blk;
    } else if (p - 8 * cls < N - 8 * n8) {
        seq = 8 * n8 + (p - 8 * cls);
    }
    rcodes[idx] = seq < N ? codes[(size_t)s * NP + seq] : 0;
    if (s == 0) rw[p] = seq < N ? w[seq] : 0.0f;
}

// Work items of lib.rs's order on f32 MFMA: an item is up to four 16x16
// sub-blocks of one 64x64 tile (`bits`), one per wave (the u-th computed
// sub-block in column-major order goes to wave u), owning the 16-row blocks
// `owned` of the tile's segments.  Per 64-position stage, lane (r, g) needs
// the dword of its a row and of its b row at 16 grp + 4 g (elements 16 grp +
// 4 e + g, e = 0..3, of the four 16-element groups grp) and the four weights
// beside them.  The candidate loop copies each wave's stage operands into a
// per-wave LDS ring by LDS-DMA (kItemStage: no barriers, the waves never wait
// for each other before the epilogue); full runs share each stage's A
// operands through LDS (kItemAShare, a barrier per stage) and copy each
// wave's B rows into a per-wave ring the same way.  Same sums, same order,
// same epilogue as pair_valu_kernel<MF, REF> (bit-identical rows).
// LOOP: the candidate launch over the screen's item list (buckets, work
// counter, fused chunk scan); else the full run's tiles in four 16-row items
// each (workgroup 4t + q: tile t's row block q).
// the item kernel's operands: byte converts of masked code dwords (per-element
// selects were 8.5% slower at C2, DESIGN Appendix A)
// byte e of x as a float by v_cvt_f32_ubyte<e> (no shift or mask first; the
// compiler's own lowering extracts the byte first).  Inline asm is invisible
// to the hazard recognizer as a VALU write: a result that an MFMA reads
// directly needs the VALU -> MFMA wait states inside the statement (NOP = 1);
// one that a VALU op consumes first (the weight products) does not.
template <int NOP>
__device__ __forceinline__ float cvt_ubyte(uint32_t x, int e) {
    float r;
    switch (e) {
    case 0:
        if (NOP) asm("v_cvt_f32_ubyte0 %0, %1\n\ts_nop 1" : "=v"(r) : "v"(x));
        else asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(r) : "v"(x));
        break;
    case 1:
        if (NOP) asm("v_cvt_f32_ubyte1 %0, %1\n\ts_nop 1" : "=v"(r) : "v"(x));
        else asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(x));
        break;
    case 2:
        if (NOP) asm("v_cvt_f32_ubyte2 %0, %1\n\ts_nop 1" : "=v"(r) : "v"(x));
        else asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(r) : "v"(x));
        break;
    default:
        if (NOP) asm("v_cvt_f32_ubyte3 %0, %1\n\ts_nop 1" : "=v"(r) : "v"(x));
        else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(r) : "v"(x));
        break;
    }
    return r;
}
#ifndef WLD_REF_ITEM_WG
#define WLD_REF_ITEM_WG 6  // workgroups per CU, full runs (<= 85 VGPRs: 72 with the shared A operands)
#endif
#ifndef WLD_REF_ITEML_WG
#define WLD_REF_ITEML_WG 5  // ... the candidate loop (<= 102 VGPRs: 75 with the LDS-staged operands)
#endif
// Full runs (not LOOP) load each stage's operands at its top instead of one
// stage ahead: 70 instead of 96 VGPRs, six workgroups per CU instead of five,
// and the co-resident waves cover the latency (C2 -2.5%, profiles/r05v/; the
// matrix pipe fills only with many waves in their sums).
// kItemAShare (full runs): the four waves of an item share its 16 rows,
// so each forms the A operands (w x in, w x major) of one 16-position group of
// a stage and writes them to LDS, and every wave reads all four: a quarter of
// the A-side converts and products per wave.  The f32 MFMA runs on the same
// ALUs as the vector instructions (tools/probes/f32_mfma_rate_probe.hip:
// ~1.5x the cycles per MFMA with the item's operand work beside it, even at
// eight waves per SIMD), so vector instructions cost MFMA throughput directly.
// C2 0.1184 -> 0.1114 ms (profiles/r05ad/; rows bit-identical, 191 tests).
constexpr bool kItemAShare = true;
// kItemStage (the candidate loop): each wave's stage operands — its 16 a rows'
// and 16 b rows' 64 code bytes and the 64 weights — copied into a per-wave
// three-slot LDS ring by LDS-DMA in whole 16-byte pieces (three copies per
// stage), then read as the MFMA operands, instead of twelve fragment-shaped
// global loads per stage (16 rows x 4 bytes per instruction) one stage
// ahead.  LD blocks: the candidate launch 0.331 -> 0.314 ms at five
// workgroups per CU (profiles/r06s/, r06t/, r06u/; four per CU: 0.318), PMC
// MFMA busy 0.551 -> 0.573 (the guide's rule for fragment-shaped operand loads)
constexpr bool kItemStage = true;
constexpr uint32_t kItemSlot = 2048 + 256;  // A 1 KB | B 1 KB | weights 256 B
template <bool LOOP>
__global__ __launch_bounds__(256, LOOP ? WLD_REF_ITEML_WG : WLD_REF_ITEM_WG) void ref_item_kernel(
    const uint8_t *__restrict__ rcodes, const float *__restrict__ rw, const uint8_t *__restrict__ site_ok,
    const uint32_t *__restrict__ tiles, uint32_t n_tiles, const uint32_t *__restrict__ tile_bits,
    unsigned *tile_work, const unsigned *tile_buckets, uint32_t bucket_cap, uint32_t L, uint32_t NPr,
    uint32_t ref_cs, uint32_t ref_tail_n, uint32_t n_chunk_rows, float thr, OrderArgs o, ScanArgs sa) {
    __shared__ unsigned long long sBits[kTile];  // compaction: passing b per a row
    __shared__ uint32_t sRowBase[kTile];
    // (full runs only: a candidate item may pack sub-blocks of several row
    // blocks, whose waves need different A operands)
    constexpr bool kAShare = kItemAShare && !LOOP;
    // (kAShare) two stages of A operands: [stage & 1][group][element][lane] (u, v)
    __shared__ float2 sAop[kAShare ? 2 * 16 * 64 : 1];
    constexpr bool kStage = kItemStage && LOOP;
    __shared__ __attribute__((aligned(16))) uint8_t sRing[kStage ? 4 * 3 * kItemSlot : 16];
    // (full runs, kAShare: each wave's B rows staged by LDS-DMA in a two-slot
    // ring instead of four fragment-shaped loads per stage; C2's launch
    // 0.111 -> 0.104 ms, profiles/r06aj/)
    __shared__ __attribute__((aligned(16))) uint8_t sBRing[kAShare ? 4 * 2 * 1024 : 16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, r = lane & 15, g = lane >> 4;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    auto compute_item = [&](uint32_t tile, uint32_t bits, uint32_t owned) {
        const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu;
        const uint32_t a0 = ta * kTile, b0 = tb * kTile;
        // this wave's sub-block: the wave-th set bit in column-major order
        uint32_t cm = 0;
        for (uint32_t k = 0; k < 16; ++k) cm |= ((bits >> (4 * (k & 3) + (k >> 2))) & 1u) << k;
        for (uint32_t t = 0; t < wave; ++t) cm &= cm - 1u;
        cm = __builtin_amdgcn_readfirstlane(cm);
        const bool has = cm != 0;
        const uint32_t kq = has ? (uint32_t)__builtin_ctz(cm) : 0u, ui = kq & 3u, un = kq >> 2;
        // lane (r, g) holds the pairs (a = 16 ui + 4 g + e, b = 16 un + r), e = 0..3
        float tot[4][4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int q = 0; q < 4; ++q) tot[e][q] = 0.0f;
        uint32_t okA4 = 0, okB = 0;  // the epilogue's site flags
        // (kAShare: a wave without a sub-block, left of a diagonal tile's
        // diagonal, still forms its share of the item's A operands and keeps
        // the stage barriers; the item's 16 rows are its row block, ctz(owned))
        if (has || kAShare) {
            const uint32_t urow = kAShare ? (uint32_t)__builtin_ctz(owned) : ui;
            const uint8_t *rowA = rcodes + (size_t)(a0 + 16 * urow + r) * NPr + 4 * g;
            const float *wg = rw + 4 * g;
            const uint32_t cls = 64 * ref_cs, n_st = 8 * ref_cs;
            uint32_t ca[4], cb[4];
            float4 cw[4];
            // the scalar tail's codes and weights (positions 8 cls .. 8 cls + 7),
            // all loaded at once after the last stage (one round trip, not one
            // per position): ca[e] / cb[e] =
            // a row e's bytes 0-3 / 4-7, cw[0], cw[1] = the weights, cw[2].x /
            // .y = the b row's bytes
            auto fetch_tail = [&] {
                const size_t p0 = 8 * (size_t)cls;
                const uint2 b8 = *reinterpret_cast<const uint2 *>(rcodes + (size_t)(b0 + 16 * un + r) * NPr + p0);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint2 a8 =
                        *reinterpret_cast<const uint2 *>(rcodes + (size_t)(a0 + 16 * ui + 4 * g + e) * NPr + p0);
                    ca[e] = a8.x, cb[e] = a8.y;
                }
                cw[0] = *reinterpret_cast<const float4 *>(rw + p0);
                cw[1] = *reinterpret_cast<const float4 *>(rw + p0 + 4);
                cw[2].x = __uint_as_float(b8.x);
                cw[2].y = __uint_as_float(b8.y);
            };
            if constexpr (kAShare) {
                // this wave's share: group `wave` of each stage (rows of the item's
                // row block, lane (r, g) its row r, elements 4 e + g)
                const uint8_t *rowAs = rowA + 16 * wave;
                const float *wgs = wg + 16 * wave;
                uint32_t sa_c = 0;
                float4 sa_w = make_float4(0.f, 0.f, 0.f, 0.f);
                auto fetch2 = [&](uint32_t k0) {
                    sa_c = *reinterpret_cast<const uint32_t *>(rowAs + k0);
                    sa_w = *reinterpret_cast<const float4 *>(wgs + k0);
                };
                // this wave's 16 b rows' 64 bytes of stage st in ring slot st & 1
                // (lane l's 16 bytes at 16 l: row l / 4, piece (l & 3) ^ ((l >> 4) & 3))
                const uint32_t bring = lds_addr(sBRing) + wave * 2 * 1024;
                const uint8_t *baseB = rcodes + (size_t)(b0 + 16 * un) * NPr;
                const uint32_t bvoff = (lane >> 2) * NPr + 16 * ((lane & 3) ^ ((lane >> 4) & 3));
                auto issueB = [&](uint32_t st) { glds16_s(baseB + 64 * st, bvoff, bring + (st & 1u) * 1024); };
                if (n_st) fetch2(0);
                if (has && n_st) issueB(0);
                v4f acc[4];
                uint32_t in_cls = 0;
                for (uint32_t st = 0; st < n_st; ++st) {
                    if (in_cls == 0)
#pragma unroll
                        for (int q = 0; q < 4; ++q) acc[q] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
                    float2 *dst = sAop + (st & 1) * 1024 + wave * 256 + lane;
                    {
                        const uint32_t ai = sa_c & 0x01010101u, am = (sa_c >> 1) & 0x01010101u;
                        const float we[4] = {sa_w.x, sa_w.y, sa_w.z, sa_w.w};
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            dst[64 * e] = make_float2(we[e] * cvt_ubyte<0>(ai, e), we[e] * cvt_ubyte<0>(am, e));
                    }
                    uint32_t B[4];
                    if (has) {  // (uniform per wave)
                        // stage st + 1's B into the slot this wave read stage st - 1
                        // from; stage st's copy (the only load outstanding here) is
                        // waited for first — the compiler waits before the asm anyway
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (st + 1 < n_st) issueB(st + 1);
                    }
                    if (st + 1 < n_st) fetch2(64 * (st + 1));
                    __syncthreads();  // the stage's four groups written (and the buffer's last readers done)
                    if (has) {
                        const uint8_t *pb = sBRing + (wave * 2 + (st & 1u)) * 1024;
#pragma unroll
                        for (int grp = 0; grp < 4; ++grp)
                            B[grp] = *reinterpret_cast<const uint32_t *>(pb + 16 * (4 * r + (grp ^ ((r >> 2) & 3))) + 4 * g);
                    }
                    const float2 *src = sAop + (st & 1) * 1024 + lane;
                    if (has)  // (uniform per wave)
#pragma unroll
                    for (int grp = 0; grp < 4; ++grp) {
                        const uint32_t bi = B[grp] & 0x01010101u, bm = (B[grp] >> 1) & 0x01010101u;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float2 uv = src[256 * grp + 64 * e];
                            const float fi = cvt_ubyte<1>(bi, e), fm = cvt_ubyte<1>(bm, e);
                            acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.x, fi, acc[0], 0, 0, 0);
                            acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.y, fi, acc[1], 0, 0, 0);
                            acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.x, fm, acc[2], 0, 0, 0);
                            acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(uv.y, fm, acc[3], 0, 0, 0);
                        }
                    }
                    if (++in_cls == ref_cs) {
                        in_cls = 0;
#pragma unroll
                        for (int e = 0; e < 4; ++e)
#pragma unroll
                            for (int q = 0; q < 4; ++q) tot[e][q] += acc[q][e];
                    }
                }
            } else if constexpr (kStage) {
                // slot s of this wave's ring: A image (lane l's 16 bytes at 16 l:
                // a row l / 4, piece (l & 3) ^ ((l >> 4) & 3) of the stage's 64
                // bytes, so the reads below hit distinct banks), B image the
                // same, then the 64 weights
                const uint32_t ring = lds_addr(sRing) + wave * 3 * kItemSlot;
                const uint8_t *baseA = rcodes + (size_t)(a0 + 16 * ui) * NPr;
                const uint8_t *baseB = rcodes + (size_t)(b0 + 16 * un) * NPr;
                const uint32_t voff = (lane >> 2) * NPr + 16 * ((lane & 3) ^ ((lane >> 4) & 3));
                auto issue = [&](uint32_t st, uint32_t slot) {
                    const uint32_t d = ring + slot * kItemSlot, k0 = 64 * st;
                    glds16_s(baseA + k0, voff, d);
                    glds16_s(baseB + k0, voff, d + 1024);
                    glds4_s(rw + k0, 4 * lane, d + 2048);
                };
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (only the ring's copies counted below)
                if (n_st) issue(0, 0);
                if (n_st > 1) issue(1, 1);
                v4f acc[4];
                uint32_t in_cls = 0, slot = 0;
                for (uint32_t st = 0; st < n_st; ++st) {
                    if (in_cls == 0)
#pragma unroll
                        for (int q = 0; q < 4; ++q) acc[q] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
                    // stage st + 2 into the slot stage st - 1 was read from (its
                    // reads done), then wait for stage st's three copies
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (st + 2 < n_st) {
                        issue(st + 2, slot == 0 ? 2u : slot - 1u);
                        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                    } else if (st + 1 < n_st) {
                        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
                    } else {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    const uint8_t *p = sRing + (wave * 3 + slot) * kItemSlot;
                    uint32_t A[4], B[4];
                    float4 Wt[4];
#pragma unroll
                    for (int grp = 0; grp < 4; ++grp) {
                        const uint32_t pos = 16 * (4 * r + (grp ^ ((r >> 2) & 3))) + 4 * g;
                        A[grp] = *reinterpret_cast<const uint32_t *>(p + pos);
                        B[grp] = *reinterpret_cast<const uint32_t *>(p + 1024 + pos);
                        Wt[grp] = *reinterpret_cast<const float4 *>(p + 2048 + 4 * (16 * grp + 4 * g));
                    }
#pragma unroll
                    for (int grp = 0; grp < 4; ++grp) {
                        const float we[4] = {Wt[grp].x, Wt[grp].y, Wt[grp].z, Wt[grp].w};
                        const uint32_t ai = A[grp] & 0x01010101u, am = (A[grp] >> 1) & 0x01010101u;
                        const uint32_t bi = B[grp] & 0x01010101u, bm = (B[grp] >> 1) & 0x01010101u;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            // w x 1.0 or w x 0.0: exact; a -0.0 term (negative w
                            // masked) adds nothing to a chain that starts at +0.0
                            const float u = we[e] * cvt_ubyte<0>(ai, e), v = we[e] * cvt_ubyte<0>(am, e);
                            const float fi = cvt_ubyte<1>(bi, e), fm = cvt_ubyte<1>(bm, e);
                            acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, fi, acc[0], 0, 0, 0);
                            acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, fi, acc[1], 0, 0, 0);
                            acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, fm, acc[2], 0, 0, 0);
                            acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, fm, acc[3], 0, 0, 0);
                        }
                    }
                    slot = slot == 2 ? 0u : slot + 1u;
                    if (++in_cls == ref_cs) {
                        in_cls = 0;
#pragma unroll
                        for (int e = 0; e < 4; ++e)
#pragma unroll
                            for (int q = 0; q < 4; ++q) tot[e][q] += acc[q][e];
                    }
                }
            }
            // the scalar tail (lib.rs:461-480), onto the horizontal sums in order
            // (ref_tail_n <= 7, uniform)
            // (one position per step: the byte queues shift down by 8 bits, the
            // weights by one register)
            // the epilogue's site flags (one dword: the lane's four a rows; one
            // byte: its b column) in the same round trip as the tail, not one
            // load per pair behind the sums
            if (has) {
            okA4 = *reinterpret_cast<const uint32_t *>(site_ok + a0 + 16 * ui + 4 * g);
            okB = site_ok[b0 + 16 * un + r];
            if (ref_tail_n) fetch_tail();
            float4 wlo = cw[0], whi = cw[1];
            uint32_t qb0 = __float_as_uint(cw[2].x), qb1 = __float_as_uint(cw[2].y);
#pragma unroll 1
            for (uint32_t t = 0; t < ref_tail_n; ++t) {
                const float we = wlo.x;
                const float fi = (float)(qb0 & 1u), fm = (float)((qb0 >> 1) & 1u);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t xa = ca[e];
                    const float u = (xa & kCodeIn) ? we : 0.0f, v = (xa & kCodeMaj) ? we : 0.0f;
                    tot[e][0] = __builtin_fmaf(u, fi, tot[e][0]);
                    tot[e][1] = __builtin_fmaf(v, fi, tot[e][1]);
                    tot[e][2] = __builtin_fmaf(u, fm, tot[e][2]);
                    tot[e][3] = __builtin_fmaf(v, fm, tot[e][3]);
                    ca[e] = (ca[e] >> 8) | (cb[e] << 24);
                    cb[e] >>= 8;
                }
                qb0 = (qb0 >> 8) | (qb1 << 24);
                qb1 >>= 8;
                wlo = make_float4(wlo.y, wlo.z, wlo.w, whi.x);
                whi = make_float4(whi.y, whi.z, whi.w, 0.0f);
            }
            }
        }
        // ---- epilogue (lib.rs:482-520, 660) --------------------------------
        uint32_t passmask = 0;  // bit e
        float res[4][3];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t al = 16 * ui + 4 * g + e, bl = 16 * un + r, a = a0 + al, b = b0 + bl;
            float d, dp, r2;
            ld_epilogue(tot[e][0], tot[e][1], tot[e][2], tot[e][3], d, dp, r2);
            res[e][0] = d;
            res[e][1] = dp;
            res[e][2] = r2;
            if (has && a < b && b < L && ((okA4 >> (8 * e)) & 0xFFu) && okB && r2 > thr) passmask |= 1u << e;
        }
        // ---- compaction: the tile's 64x64 pass bits, rows in b order ---------
        const bool own_row = tid < kTile && ((owned >> (tid >> 4)) & 1u);
        const uint32_t quarters = (uint32_t)__popc(owned);
        if (!__syncthreads_or(passmask != 0)) {
            if (own_row) o.seg_cnt[(size_t)(a0 + tid) * o.T + tb] = 0;
            if (tid == 0) tile_done(o, ta, tb, n_chunk_rows, quarters);
            return;
        }
        if (tid < kTile) sBits[tid] = 0ull;
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (passmask & (1u << e)) atomicOr(&sBits[16 * ui + 4 * g + e], 1ull << (16 * un + r));
        __syncthreads();
        if (tid < kTile) {
            const uint32_t row = tid;
            const uint32_t cnt = __popcll(sBits[row]);
            const uint32_t incl = wave_inclusive_scan(cnt);
            const uint32_t excl = incl - cnt;
            const uint32_t total = __shfl(incl, 63, 64);
            unsigned long long base = 0;
            if (row == 63 && total) base = atomicAdd(o.cursor, (unsigned long long)total);
            base = __shfl(base, 63, 64);
            sRowBase[row] = (uint32_t)base + excl;
            if (own_row) {  // (a row outside the item's blocks has no pass: cnt 0)
                o.seg_cnt[(size_t)(a0 + row) * o.T + tb] = (uint8_t)cnt;
                o.seg_off[(size_t)(a0 + row) * o.T + tb] = (uint32_t)base + excl;
            }
            if (row == 63 && total)
                atomicAdd(&o.chunk_total[chunk_linear(n_chunk_rows, ta / kTilesPerChunk, tb / kTilesPerChunk)], total);
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (!(passmask & (1u << e))) continue;
            const uint32_t al = 16 * ui + 4 * g + e, bl = 16 * un + r;
            const uint64_t pos = (uint64_t)sRowBase[al] + __popcll(sBits[al] & ((1ull << bl) - 1ull));
            if (pos < o.st_capacity) {
                o.st_a[pos] = a0 + al;
                o.st_b[pos] = b0 + bl;
                o.st_d[pos] = res[e][0];
                o.st_dp[pos] = res[e][1];
                o.st_r2[pos] = res[e][2];
            }
        }
        if (tid == 0) tile_done(o, ta, tb, n_chunk_rows, quarters);
    };

    if constexpr (!LOOP) {
        const uint32_t tile = tiles[blockIdx.x >> 2], q = blockIdx.x & 3;
        // a diagonal tile's sub-blocks left of row block q's diagonal one hold
        // only pairs a > b: not computed (their waves idle to the epilogue)
        const uint32_t cols = (tile >> 16) == (tile & 0xFFFFu) ? 0xFu & ~((1u << q) - 1u) : 0xFu;
        if (tile != kNoTile) compute_item(tile, cols << (4 * q), 1u << q);  // kNoTile: padding of an XCD-ordered list
        scan_tail(sa, gridDim.x);  // (every workgroup takes a ticket when the scan is fused)
    } else {
        // the screen's items, heaviest bucket first; the first by workgroup id
        // (rounds dealt in snake order, heavy beside light on a CU), the next
        // from the work counter (zeroed by the screen); every entry and its
        // tile checked before anything is read through them
        __shared__ uint32_t s_next, s_pre[17];
        cand_prefix(tile_buckets, s_pre);
        const uint32_t nt = s_pre[16];
        uint32_t first = blockIdx.x;
        {
            constexpr uint32_t R = WLD_REF_ITEML_WG;
            const uint32_t m = gridDim.x / R, k = m ? blockIdx.x / m : R, j = blockIdx.x - (k < R ? k * m : 0u);
            if (k < R) first = (k & 1) ? (k + 1) * m - 1 - j : k * m + j;
        }
        for (uint32_t bi = first; bi < nt;) {
            const uint32_t e = cand_entry_checked(o, s_pre, bucket_cap, bi);
            const uint32_t tile = e != ~0u ? tiles[e] : kNoTile;
            const uint32_t bits = e != ~0u ? tile_bits[e] : 0u;
            uint32_t owned = 0;
            for (uint32_t q = 0; q < 4; ++q) owned |= ((bits >> (4 * q)) & 0xFu) ? 1u << q : 0u;
            if (tile_in_range(tile, L) && bits && __popc(bits) <= 4)
                compute_item(tile, bits, owned);
            else if (e != ~0u && threadIdx.x == 0)
                report_guard(o, kGuardTile);
            if (threadIdx.x == 0) s_next = gridDim.x + atomicAdd(tile_work, 1u);
            __syncthreads();  // (also: the next item's compaction reuses the LDS)
            bi = s_next;
            __syncthreads();
        }
        scan_tail(sa, nt, false, first);
    }
}

// One class chain of lib.rs's four sums (lib.rs:416-480) over positions
// [q0, q1) of the lane-class layout, in element order: adds of selected
// weights, lib.rs's select + add.  A 16-position group holds element 4j + g at
// position 4g + j, so a 16-byte read gives 16 elements, taken in element order
// from its dwords.  The next group's loads are issued before this group's
// adds (a chain walks ~2,000 sequences of two random site rows).
__device__ inline void ref_chain(const uint8_t *ra, const uint8_t *rb, const float *rw, uint32_t q0, uint32_t q1,
                                 float (&acc)[4]) {
    if (q0 >= q1) return;
    uint4 va = *reinterpret_cast<const uint4 *>(ra + q0), vb = *reinterpret_cast<const uint4 *>(rb + q0);
    float4 w0 = *reinterpret_cast<const float4 *>(rw + q0), w1 = *reinterpret_cast<const float4 *>(rw + q0 + 4);
    float4 w2 = *reinterpret_cast<const float4 *>(rw + q0 + 8), w3 = *reinterpret_cast<const float4 *>(rw + q0 + 12);
    for (uint32_t q = q0; q < q1; q += 16) {
        const uint32_t A[4] = {va.x, va.y, va.z, va.w}, B[4] = {vb.x, vb.y, vb.z, vb.w};
        const float W[16] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w,
                             w2.x, w2.y, w2.z, w2.w, w3.x, w3.y, w3.z, w3.w};
        if (q + 16 < q1) {
            va = *reinterpret_cast<const uint4 *>(ra + q + 16);
            vb = *reinterpret_cast<const uint4 *>(rb + q + 16);
            w0 = *reinterpret_cast<const float4 *>(rw + q + 16);
            w1 = *reinterpret_cast<const float4 *>(rw + q + 20);
            w2 = *reinterpret_cast<const float4 *>(rw + q + 24);
            w3 = *reinterpret_cast<const float4 *>(rw + q + 28);
        }
        // per dword: the "in" and "major" bits of its 4 bytes as 0/1 bytes,
        // each turned into 0.0/1.0 by a byte convert; u = in_a w, v = maj_a w
        // (exact), then fmaf(u, f_b, acc) = acc + u f_b rounded once, as
        // lib.rs's select + add (finite weights: this path follows the i8
        // pass, which needs them)
        uint32_t ai[4], am[4], bi[4], bm[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            ai[g] = A[g] & 0x01010101u;
            am[g] = (A[g] >> 1) & 0x01010101u;
            bi[g] = B[g] & 0x01010101u;
            bm[g] = (B[g] >> 1) & 0x01010101u;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int g = e & 3, j = e >> 2;  // element 4j + g at position 4g + j
            const float we = W[4 * g + j];
            const float u = (float)((ai[g] >> (8 * j)) & 0xFFu) * we, v = (float)((am[g] >> (8 * j)) & 0xFFu) * we;
            const float fi = (float)((bi[g] >> (8 * j)) & 0xFFu), fm = (float)((bm[g] >> (8 * j)) & 0xFFu);
            acc[0] = __builtin_fmaf(u, fi, acc[0]);
            acc[1] = __builtin_fmaf(v, fi, acc[1]);
            acc[2] = __builtin_fmaf(u, fm, acc[2]);
            acc[3] = __builtin_fmaf(v, fm, acc[3]);
        }
    }
}

// ... the scalar tail (lib.rs:461-480), added onto the horizontal sums
__device__ inline void ref_tail(const RefRowsLaunch &r, const uint8_t *ra, const uint8_t *rb, float (&tot)[4]) {
    for (uint32_t t = 0; t < r.ref_tail_n; ++t) {
        const uint32_t p = 8 * r.ref_cls + t;
        const uint32_t xa = ra[p], xb = rb[p];
        const float we = r.rw[p];
        const float u = (xa & kCodeIn) ? we : 0.0f, v = (xa & kCodeMaj) ? we : 0.0f;
        tot[0] += (xb & kCodeIn) ? u : 0.0f;
        tot[1] += (xb & kCodeIn) ? v : 0.0f;
        tot[2] += (xb & kCodeMaj) ? u : 0.0f;
        tot[3] += (xb & kCodeMaj) ? v : 0.0f;
    }
}

// Every staged candidate row (the staging cursor the candidate pass left):
// lib.rs's sums and epilogue, the values written back into the row's staging
// slot; whether it passes (r2 > thr) is read back from that r2 by
// ref_compact_kernel.  Up to an eighth of the grid's threads in rows, each
// row on 8 lanes, one class chain each, folded in order ((((0 + l0) + l1) +
// ...) + l7) with shuffles (8x shorter chains); more rows, one lane per row
// walking the 8 chains (no exchange), grid-stride.
__global__ __launch_bounds__(256) void ref_sums_kernel(RefRowsLaunch r, OrderArgs o) {
    const uint64_t n = min((uint64_t)*o.cursor, o.st_capacity);  // (an overflowing pass re-runs)
    const uint64_t threads = (uint64_t)gridDim.x * 256, gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t cls = r.ref_cls;
    // a staged pair outside a < b < L is not read through (kGuardPair)
    auto pair_ok = [&](uint32_t a, uint32_t b) {
        const bool ok = a < b && b < o.L;
        if (!ok) report_guard(o, kGuardPair);
        return ok;
    };
    if (n * 8 <= threads) {
        const uint64_t i = gid >> 3;
        if (i >= n) return;  // (a row's 8 lanes leave together)
        const uint32_t c = (uint32_t)(gid & 7);
        const uint32_t sa = o.st_a[i], sb = o.st_b[i];
        if (!pair_ok(sa, sb)) return;  // (the row's 8 lanes alike)
        const uint8_t *ra = r.rcodes + (size_t)sa * r.NPr, *rb = r.rcodes + (size_t)sb * r.NPr;
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f}, tot[4];
        ref_chain(ra, rb, r.rw, c * cls, (c + 1) * cls, acc);
        const int first = (int)(threadIdx.x & 63) & ~7;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float t = 0.0f;
            for (int k = 0; k < 8; ++k) t += __shfl(acc[q], first + k, 64);
            tot[q] = cls ? t : 0.0f;
        }
        if (c != 0) return;
        ref_tail(r, ra, rb, tot);
        float d, dp, r2;
        ld_epilogue(tot[0], tot[1], tot[2], tot[3], d, dp, r2);
        o.st_d[i] = d;
        o.st_dp[i] = dp;
        o.st_r2[i] = r2;
        return;
    }
    for (uint64_t i = gid; i < n; i += threads) {
        const uint32_t sa = o.st_a[i], sb = o.st_b[i];
        if (!pair_ok(sa, sb)) continue;
        const uint8_t *ra = r.rcodes + (size_t)sa * r.NPr, *rb = r.rcodes + (size_t)sb * r.NPr;
        float tot[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        for (uint32_t k = 0; k < (cls ? 8u : 0u); ++k) {
            float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            ref_chain(ra, rb, r.rw, k * cls, (k + 1) * cls, acc);
#pragma unroll
            for (int q = 0; q < 4; ++q) tot[q] += acc[q];
        }
        ref_tail(r, ra, rb, tot);
        float d, dp, r2;
        ld_epilogue(tot[0], tot[1], tot[2], tot[3], d, dp, r2);
        o.st_d[i] = d;
        o.st_dp[i] = dp;
        o.st_r2[i] = r2;
    }
}

// One wave per tile slice (wave-strided over the slices): the rows with r2 >
// thr (lib.rs:660, strict; every staged pair is valid) move down in place,
// 64 at a time — a row's new position never exceeds its old one and a batch
// is read before it is written — so
// the slice keeps its (a, b) order; then the tile's 64 segment counts/offsets
// are rewritten and the dropped rows leave its chunk total.  The run's chunk
// scan runs in the last workgroup.
__global__ __launch_bounds__(256) void ref_compact_kernel(RefRowsLaunch r, OrderArgs o) {
    __shared__ uint32_t sCnt[4][kTile];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t *cnt = sCnt[wv];
    const uint32_t ns = *r.slice_count;
    for (uint32_t si = 4 * blockIdx.x + wv; si < ns;) {
        const uint32_t base = r.slices[3 * si], total = r.slices[3 * si + 1], tile = r.slices[3 * si + 2];
        const uint32_t ta = tile >> 16, tb = tile & 0xFFFFu, a0 = ta * kTile;
        if (!tile_in_range(tile, o.L) || total > kTile * kTile) {
            if (lane == 0) report_guard(o, kGuardSlice);
        } else if ((uint64_t)base + total <= o.st_capacity) {  // else not stored: the pass re-runs
            cnt[lane] = 0;
            uint32_t kept = 0;
            for (uint32_t c0 = 0; c0 < total; c0 += 64) {
                const uint32_t i = base + c0 + lane;
                const bool in = c0 + lane < total;
                const uint32_t a = in ? o.st_a[i] : 0u, b = in ? o.st_b[i] : 0u;
                const float d = in ? o.st_d[i] : 0.0f, dp = in ? o.st_dp[i] : 0.0f, r2 = in ? o.st_r2[i] : 0.0f;
                const bool pass = in && r2 > r.thr;
                const uint64_t bal = __ballot(pass);
                if (pass) {
                    const uint32_t pos = base + kept + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
                    o.st_a[pos] = a;
                    o.st_b[pos] = b;
                    o.st_d[pos] = d;
                    o.st_dp[pos] = dp;
                    o.st_r2[pos] = r2;
                    atomicAdd(&cnt[a - a0], 1u);
                }
                kept += (uint32_t)__popcll(bal);
            }
            // the slice is in (a, b) order: a's rows follow the smaller a's
            const uint32_t c = cnt[lane], incl = wave_inclusive_scan(c);
            o.seg_cnt[(size_t)(a0 + lane) * o.T + tb] = (uint8_t)c;
            o.seg_off[(size_t)(a0 + lane) * o.T + tb] = base + incl - c;
            if (lane == 0 && kept < total)
                atomicSub(&o.chunk_total[chunk_linear(r.n_chunk_rows, ta / kTilesPerChunk, tb / kTilesPerChunk)],
                          total - kept);
        }
        // the tile is finished now (per-chunk progress: its candidates are
        // summed and compacted; tile_epilogue left it to this kernel)
        if (lane == 0 && tile_in_range(tile, o.L)) tile_done(o, ta, tb, r.n_chunk_rows);
        si += 4 * gridDim.x;  // (static: tens of thousands of small slices would queue on one work counter)
    }
    // every wave's atomics (chunk totals) are drained before the ticket
    scan_tail(r.scan, (ns + 3) / 4, true);
}

void launch_ref_rows(const RefRowsLaunch &r, const OrderArgs &o, hipStream_t s) {
    hipLaunchKernelGGL(ref_sums_kernel, dim3(kRefRowsGrid), dim3(256), 0, s, r, o);
    hipLaunchKernelGGL(ref_compact_kernel, dim3(kRefRowsGrid), dim3(256), 0, s, r, o);
}

void ref_layout_dims(size_t N, uint32_t *cls, uint32_t *tail, size_t *NPr) {
    const size_t stages = (N / 8 + 63) / 64;  // 64-sequence stages per lane class (0 when N < 8)
    *cls = (uint32_t)(stages * 64);
    *tail = (N % 8) ? 1u : 0u;
    *NPr = 8 * (size_t)*cls + (*tail ? 64 : 0);
    if (*NPr == 0) *NPr = 64;  // N == 0: one all-padding stage (a tail stage: T = 0, every pair NaN)
}

void launch_ref_layout(const uint8_t *codes, const float *w_pad, size_t LP, size_t NP, size_t N, uint8_t *rcodes,
                       float *rw, hipStream_t s) {
    uint32_t cls, tail;
    size_t NPr;
    ref_layout_dims(N, &cls, &tail, &NPr);
    const size_t n = LP * NPr;
    hipLaunchKernelGGL(ref_layout_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, codes, w_pad,
                       (uint32_t)LP, (uint32_t)NP, (uint32_t)N, (uint32_t)NPr, cls, rcodes, rw);
}

namespace {
template <bool DENSE, bool SAFE, bool MF, bool REF, bool LOOP>
void launch_v(const ValuLaunch &v, uint32_t grid, uint32_t flush, uint32_t cs, const OrderArgs &o,
              const DenseArgs &dn, hipStream_t s) {
    hipLaunchKernelGGL((pair_valu_kernel<DENSE, SAFE, MF, REF, LOOP>), dim3(grid), dim3(256), 0, s, v.codes, v.w,
                       v.site_ok, v.tiles, v.n_tiles, v.tile_count, v.tile_bits, v.tile_work, v.tile_buckets,
                       v.bucket_cap, v.L, v.NP, flush, cs, v.ref_tail_n, v.n_chunk_rows, v.thr, o, dn, v.scan);
}
}  // namespace

bool launch_pair_valu(const ValuLaunch &v, const OrderArgs &o, const DenseArgs *dense, hipStream_t s) {
    const DenseArgs dn = dense ? *dense : DenseArgs{nullptr, nullptr, nullptr, nullptr};
    const uint32_t flush = (uint32_t)std::max(1.0, std::floor(std::sqrt((double)v.NP) / 64.0 + 0.5));
    const uint32_t grid = v.tile_count ? std::min<uint32_t>(v.n_tiles, v.ref ? kRefCandidateGrid : kCandidateGrid)
                                       : v.n_tiles;
    if (grid == 0) return false;
    if (v.ref) {
        // the reference's f32 order: f32-input MFMA for finite weights, the
        // select loop otherwise (both sequential fmaf/add chains per block)
        const uint32_t cs = v.ref_cls / 64;
        if (dense) {
            if (v.safe) launch_v<true, true, false, true, false>(v, grid, flush, cs, o, dn, s);
            else launch_v<true, false, true, true, false>(v, grid, flush, cs, o, dn, s);
        } else if (v.tile_count) {
            if (v.safe) launch_v<false, true, false, true, true>(v, grid, flush, cs, o, dn, s);
            else if (v.rb_items)  // items of <= 4 sub-blocks, one per wave
                hipLaunchKernelGGL(ref_item_kernel<true>, dim3(std::min<uint32_t>(4 * v.n_tiles, kRefItemGrid)),
                                   dim3(256), 0, s, v.codes, v.w, v.site_ok, v.tiles, v.n_tiles, v.tile_bits,
                                   v.tile_work, v.tile_buckets, v.bucket_cap, v.L, v.NP, cs, v.ref_tail_n,
                                   v.n_chunk_rows, v.thr, o, v.scan);
            else launch_v<false, false, true, true, true>(v, grid, flush, cs, o, dn, s);
        } else {
            // every tile of the run: with fewer tiles than four rounds of
            // resident workgroups (BASELINE config 2: 528 tiles), each tile's
            // four 16-row blocks are separate work items (f32 MFMA path)
            if (v.safe) launch_v<false, true, false, true, false>(v, grid, flush, cs, o, dn, s);
            else if (v.n_tiles <= 4 * kRefCandidateGrid) {
                // (the run's chunk scan in the last workgroup when given)
                hipLaunchKernelGGL(ref_item_kernel<false>, dim3(4 * grid), dim3(256), 0, s, v.codes, v.w, v.site_ok,
                                   v.tiles, v.n_tiles, nullptr, nullptr, nullptr, 0u, v.L, v.NP, cs, v.ref_tail_n,
                                   v.n_chunk_rows, v.thr, o, v.scan);
                return v.scan.ticket != nullptr;
            }
            else launch_v<false, false, true, true, false>(v, grid, flush, cs, o, dn, s);
        }
        return false;
    }
    // finite weights: products and sums on the matrix cores (plain, option
    // WLD_OPT_VALU_PLAIN: the VALU loop, for A/B); non-finite weights keep the
    // select loop
    if (dense) {
        if (v.safe) launch_v<true, true, false, false, false>(v, grid, flush, 1, o, dn, s);
        else if (v.plain) launch_v<true, false, false, false, false>(v, grid, flush, 1, o, dn, s);
        else launch_v<true, false, true, false, false>(v, grid, flush, 1, o, dn, s);
    } else {
        if (v.safe) launch_v<false, true, false, false, false>(v, grid, flush, 1, o, dn, s);
        else if (v.plain) launch_v<false, false, false, false, false>(v, grid, flush, 1, o, dn, s);
        else launch_v<false, false, true, false, false>(v, grid, flush, 1, o, dn, s);
    }
    return false;
}

}  // namespace wld
