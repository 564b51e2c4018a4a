// apply_t64.hip -- the k_gf_apply instances for 64-thread workgroups (see apply.hpp).
#include "apply.hpp"
#include "apply_launch.inc"

namespace ecx {
template void launch_shape_t<64>(const Shape &, dim3, size_t, hipStream_t, const ApplyArgs &);
}  // namespace ecx
