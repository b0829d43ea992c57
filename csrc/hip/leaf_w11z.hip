// Leaf instantiations: 1 wave of 1 row per lane per participant, the zero-pivot rule
// (csrc/hip/leaf.h; split per variant so they compile in parallel).
#include "leaf.h"

#include "gelim/internal.h"

namespace gelim {
namespace big {
namespace leafk {
GELIM_LEAF_SHAPE_DEFINE(1, 1, 0)
}  // namespace leafk
}  // namespace big
}  // namespace gelim
