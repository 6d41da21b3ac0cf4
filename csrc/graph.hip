// Device neighbour sampling for the federated GNN (gfx950).
//
// One thread per frontier row (client k, node v). If client k may expand v (v is k's training
// node, or a validation node), the thread streams v's in-neighbour list and keeps the `fanout`
// entries with the smallest hash keys key(p) = hmix(hmix(hmix(hmix(seed) + client) + v) + p),
// ties to the lower position, in a register-resident sorted list. This is sampling without
// replacement with the same selection and order as `sample_neighbors_torch` in
// data/graph.py, so results do not depend on the device, the rank layout or the cohort order.
// Output: [n][fanout] neighbour ids (-1 padding), per-row counts.
#include "common.h"
#include "dls.h"

namespace {

__device__ __forceinline__ unsigned long long hmix(unsigned long long h) {
  h &= 0x7FFFFFFFull;
  h ^= h >> 16;
  h = (h * 0x45D9F3Bull) & 0x7FFFFFFFull;
  h ^= h >> 16;
  h = (h * 0x45D9F3Bull) & 0x7FFFFFFFull;
  return h ^ (h >> 16);
}

template <int MAXF>
__global__ void __launch_bounds__(256) neighbor_sample_kernel(const int* __restrict__ rowptr, const int* __restrict__ col,
                                                              const int* __restrict__ owner,
                                                              const uint8_t* __restrict__ is_val,
                                                              const int64_t* __restrict__ nodes,
                                                              const int64_t* __restrict__ clients, int n, int fanout,
                                                              unsigned long long seed_h, int* __restrict__ out_nbr,
                                                              int* __restrict__ out_cnt) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t v = nodes[t];
  const int64_t c = clients[t];
  int cnt = 0;
  unsigned key_k[MAXF];
  int key_p[MAXF];
  int base = 0;
  if (owner[v] == (int)c || is_val[v]) {
    base = rowptr[v];
    const int deg = rowptr[v + 1] - base;
    const unsigned long long hv = hmix(hmix(seed_h + (unsigned long long)c) + (unsigned long long)v);
    for (int p = 0; p < deg; ++p) {
      const unsigned key = (unsigned)hmix(hv + (unsigned long long)p);
      if (cnt == fanout && key >= key_k[cnt - 1]) continue;  // equal key: the earlier position wins
      int i = cnt < fanout ? cnt++ : fanout - 1;
      while (i > 0 && key_k[i - 1] > key) {
        key_k[i] = key_k[i - 1];
        key_p[i] = key_p[i - 1];
        --i;
      }
      key_k[i] = key;
      key_p[i] = p;
    }
  }
  int* out = out_nbr + (long)t * fanout;
  for (int i = 0; i < fanout; ++i) out[i] = i < cnt ? col[base + key_p[i]] : -1;
  out_cnt[t] = cnt;
}

}  // namespace

void neighbor_sample(const int* rowptr, const int* col, const int* owner, const uint8_t* is_val, const int64_t* nodes,
                     const int64_t* clients, int n, int fanout, unsigned long long seed_h, int* out_nbr, int* out_cnt,
                     hipStream_t s) {
  if (n <= 0) return;
  const dim3 grid(cdiv(n, 256)), block(256);
  if (fanout <= 8)
    hipLaunchKernelGGL(neighbor_sample_kernel<8>, grid, block, 0, s, rowptr, col, owner, is_val, nodes, clients, n,
                       fanout, seed_h, out_nbr, out_cnt);
  else if (fanout <= 16)
    hipLaunchKernelGGL(neighbor_sample_kernel<16>, grid, block, 0, s, rowptr, col, owner, is_val, nodes, clients, n,
                       fanout, seed_h, out_nbr, out_cnt);
  else
    hipLaunchKernelGGL(neighbor_sample_kernel<32>, grid, block, 0, s, rowptr, col, owner, is_val, nodes, clients, n,
                       fanout, seed_h, out_nbr, out_cnt);
}
