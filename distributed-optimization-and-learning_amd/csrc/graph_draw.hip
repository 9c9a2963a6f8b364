// graph_draw.hip — a fresh Erdos-Renyi mixing matrix per round, drawn on the device.
//
// BASELINE config 5 mixes with a time-varying dense W: every round a new
// undirected G(n, p) adjacency A under the reference's 'stochastic' weighting
// (DIST/simulators.py:65-70: G = R o A, G /= colsum(G), W = G^T).  The torch
// form (graph.erdos_renyi_stochastic) takes nine elementwise / reduction
// kernels over n^2 entries; here one kernel writes W directly:
//   * row j of W is column j of G, so its normaliser colsum_j is the sum of
//     the row's own entries: one workgroup per row computes the n entries
//     g_ij = R_ij [i != j] [U_{min(i,j),max(i,j)} < p] from a counter-based
//     hash (no random state in memory), reduces them in a fixed order, and
//     writes g_ij / colsum_j (0 where the entry is 0 or the column is empty,
//     as the reference's Neighbors drops NaN / <= 0 weights);
//   * U is keyed by the unordered pair, so A is symmetric by construction.
// Bytes: n^2 * 4 written once (HBM-bound store stream), nothing read.
// The draw is a synthetic workload (not a reference topology): seeded and
// deterministic, but not the torch generator's stream.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dol_hip.h"
#include "dol_common.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ uint32_t mix32(uint32_t x) {  // 32-bit integer hash (two multiplies)
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// uniform in [0, 1) with 24 random bits (exact in fp32) for entry `idx` of stream `key`
__device__ __forceinline__ float u01(uint32_t key, uint32_t idx) {
  return float(mix32(idx * 0x9e3779b9u + key) >> 8) * (1.0f / 16777216.0f);
}

struct ErKeys {
  uint32_t edge, weight;  // per-draw stream keys (from the 64-bit seed on the host)
  uint32_t n;
  float p;
};

// g_ij of G = R o A (row i, column j)
__device__ __forceinline__ float g_entry(const ErKeys& k, uint32_t i, uint32_t j) {
  if (i == j) return 0.f;
  const uint32_t a = i < j ? i : j, b = i < j ? j : i;
  const bool edge = u01(k.edge, a * k.n + b) < k.p;
  return edge ? u01(k.weight, i * k.n + j) : 0.f;
}

// one workgroup per row j of W (= column j of G)
__global__ __launch_bounds__(kThreads) void er_stochastic_kernel(float* __restrict__ W, int64_t ldw, ErKeys k) {
  __shared__ float part[kThreads];
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  float s = 0.f;
  for (uint32_t i = t; i < k.n; i += kThreads) s += g_entry(k, i, j);
  part[t] = s;
  __syncthreads();
#pragma unroll
  for (int w = kThreads / 2; w > 0; w >>= 1) {  // fixed-order tree: deterministic colsum
    if (t < uint32_t(w)) part[t] += part[t + w];
    __syncthreads();
  }
  const float colsum = part[0];
  float* row = W + int64_t(j) * ldw;
  for (uint32_t i = t; i < k.n; i += kThreads) {
    const float g = g_entry(k, i, j);
    const float w = g / colsum;  // colsum == 0 only when every g is 0: 0/0 = NaN -> 0 below
    __builtin_nontemporal_store(w > 0.f ? w : 0.f, row + i);
  }
}

}  // namespace

extern "C" int dol_er_stochastic_f32(float* W, int64_t ldw, int32_t n, float p, uint64_t seed, hipStream_t s) {
  DOL_DIMS_OK("dol_er_stochastic_f32", ldw);
  using dol::fail;
  if (n < 0) return fail(DOL_EINVAL, "dol_er_stochastic_f32: negative size");
  if (n == 0) return DOL_OK;
  if (!W) return fail(DOL_EINVAL, "dol_er_stochastic_f32: null W");
  if (ldw < n) return fail(DOL_EINVAL, "dol_er_stochastic_f32: ldw < n");
  if (!(p >= 0.f && p <= 1.f)) return fail(DOL_EINVAL, "dol_er_stochastic_f32: p outside [0, 1]");
  if (n > 65535) return fail(DOL_EINVAL, "dol_er_stochastic_f32: n > 65535 (32-bit entry index)");
  auto splitmix = [](uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  };
  const uint64_t h = splitmix(seed);
  ErKeys k;
  k.edge = static_cast<uint32_t>(h);
  k.weight = static_cast<uint32_t>(h >> 32) ^ 0x5bd1e995u;
  k.n = static_cast<uint32_t>(n);
  k.p = p;
  hipLaunchKernelGGL(er_stochastic_kernel, dim3(static_cast<unsigned>(n)), dim3(kThreads), 0, s, W, ldw, k);
  return dol::check_launch("dol_er_stochastic_f32");
}
