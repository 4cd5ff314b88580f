// Selection kernels for k-step count 1 (d + 1 <= 16): one TU per count so the
// instances build in parallel.
#include "knn_select.hpp"

namespace mepol {
namespace knn {
template void launch_select<1>(const SelectArgs& a, hipStream_t st);
}  // namespace knn
}  // namespace mepol
