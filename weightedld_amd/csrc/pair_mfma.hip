// Placeholder until the i8 MFMA pair kernel lands (next milestone).
#include "pair_common.hpp"

namespace wld {
bool mfma_supported() { return false; }
void launch_mfma_prep(const uint8_t *, const float *, size_t, size_t, int, int8_t *, hipStream_t) {}
void launch_pair_mfma(const uint8_t *, const int8_t *, const uint8_t *, const uint32_t *, uint32_t, uint32_t, uint32_t,
                      uint32_t, float, int, const OrderArgs &, const DenseArgs *, hipStream_t) {}
}  // namespace wld
