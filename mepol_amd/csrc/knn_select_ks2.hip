// Selection kernels for k-step count 2 (d + 1 <= 32): one TU per count so the
// instances build in parallel.
#include "knn_select.hpp"

namespace mepol {
namespace knn {
template void launch_select<2>(const SelectArgs& a, hipStream_t st);
}  // namespace knn
}  // namespace mepol
