// CSR transpose of the k-NN table for the entropy gradient (the scatter of policy_update's
// autograd through iw[indices[:, :-1]], src/algorithms/mepol.py:148 / :278).
//
// For every owned candidate id j in [col_offset, col_offset + ncand): the list of query rows
// i whose first k neighbours contain j.  Built once per epoch (indices are fixed within an
// epoch) with a stable rocPRIM radix sort of (j, i) pairs, so every list has a fixed order and
// gamma_j = sum_{i in list(j)} g_i is bitwise reproducible.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace mepol {
namespace csr {

// keys[e] = local j or the sentinel ncand (entries owned by another rank); vals[e] = row id.
__global__ void make_pairs_kernel(const int32_t* __restrict__ idxT, int64_t nq, int k,
                                  int64_t col_offset, int64_t ncand, int64_t row_offset,
                                  uint32_t* __restrict__ keys, int32_t* __restrict__ vals) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nq * (int64_t)k) return;
  const int64_t j = (int64_t)idxT[e] - col_offset;  // idxT is [>=k][nq]: first k rows contiguous
  const bool own = j >= 0 && j < ncand;
  keys[e] = own ? (uint32_t)j : (uint32_t)ncand;
  vals[e] = (int32_t)(row_offset + e % nq);
}

// off[j] = number of sorted keys < j, j = 0..ncand (lower bound by binary search): the row
// offsets of the CSR straight from the sorted keys, no per-candidate counters (the former
// atomic count + single-block scan took ~0.6 ms per epoch at C3).
__global__ __launch_bounds__(256) void offsets_kernel(const uint32_t* __restrict__ keys,
                                                      int64_t ne, int64_t ncand,
                                                      int32_t* __restrict__ off) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j > ncand) return;
  int64_t lo = 0, hi = ne;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)keys[mid] < j)
      lo = mid + 1;
    else
      hi = mid;
  }
  off[j] = (int32_t)lo;
}

struct Layout {
  size_t keys_in, keys_out, vals_in, temp, temp_bytes, total;
};

static int layout(int64_t nq, int k, int64_t ncand, Layout* L) {
  const int64_t ne = nq * (int64_t)k;
  size_t temp = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (uint32_t*)nullptr,
                                                    (uint32_t*)nullptr, (int32_t*)nullptr,
                                                    (int32_t*)nullptr, (int)std::max<int64_t>(ne, 1));
  if (e != hipSuccess) {
    set_error("mepol_csr: radix sort size query failed: %s", hipGetErrorString(e));
    return (int)e;
  }
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  const size_t nb = (size_t)std::max<int64_t>(ne, 1) * 4;
  L->keys_in = take(nb);
  L->keys_out = take(nb);
  L->vals_in = take(nb);
  L->temp = take(temp);
  L->temp_bytes = temp;
  L->total = off;
  return 0;
}

}  // namespace csr
}  // namespace mepol

using namespace mepol;
using namespace mepol::csr;

extern "C" int mepol_csr_workspace_size(int64_t nq, int k, int64_t ncand, size_t* bytes) {
  if (nq < 0 || k <= 0 || ncand <= 0 || ncand >= (1ll << 31) || !bytes) {
    set_error("mepol_csr_workspace_size: bad arguments");
    return kErrBadArg;
  }
  Layout L;
  int rc = layout(nq, k, ncand, &L);
  if (rc) return rc;
  *bytes = L.total;
  return 0;
}

extern "C" int mepol_csr_build(const int32_t* idxT, int64_t nq, int k, int64_t col_offset,
                               int64_t ncand, int64_t row_offset, int32_t* csr_off,
                               int32_t* csr_rows, void* workspace, size_t workspace_bytes,
                               void* stream) {
  if (!idxT || !csr_off || !csr_rows || !workspace || k <= 0 || ncand <= 0 || nq < 0) {
    set_error("mepol_csr_build: bad arguments");
    return kErrBadArg;
  }
  Layout L;
  int rc = layout(nq, k, ncand, &L);
  if (rc) return rc;
  if (workspace_bytes < L.total) {
    set_error("mepol_csr_build: workspace %zu < %zu bytes", workspace_bytes, L.total);
    return kErrWorkspace;
  }
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  uint32_t* keys_in = (uint32_t*)(ws + L.keys_in);
  uint32_t* keys_out = (uint32_t*)(ws + L.keys_out);
  int32_t* vals_in = (int32_t*)(ws + L.vals_in);
  const int64_t ne = nq * (int64_t)k;
  if (ne > 0) {
    hipLaunchKernelGGL(make_pairs_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st,
                       idxT, nq, k, col_offset, ncand, row_offset, keys_in, vals_in);
    MEPOL_CHECK_LAUNCH();
    int end_bit = 1;
    while ((1ll << end_bit) <= ncand) ++end_bit;
    size_t temp = L.temp_bytes;
    MEPOL_HIP(hipcub::DeviceRadixSort::SortPairs(ws + L.temp, temp, keys_in, keys_out, vals_in,
                                                 csr_rows, (int)ne, 0, end_bit, st));
  }
  hipLaunchKernelGGL(offsets_kernel, dim3((unsigned)((ncand + 1 + 255) / 256)), dim3(256), 0, st,
                     keys_out, ne, ncand, csr_off);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
