// Selection kernels for k-step count 3 (d + 1 <= 48): one TU per count so the
// instances build in parallel.
#include "knn_select.hpp"

namespace mepol {
namespace knn {
template void launch_select<3>(const SelectArgs& a, hipStream_t st);
}  // namespace knn
}  // namespace mepol
