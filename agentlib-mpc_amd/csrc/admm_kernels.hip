// admm_kernels.hip — agent-batched ADMM arithmetic (consensus and exchange).
//
// Reference semantics: ConsensusVariable / ExchangeVariable
// (agentlib_mpc/data_structures/admm_datatypes.py:217-331), ADMM._set_mean_coupling_values
// and update_lambda (modules/dmpc/admm/admm.py:528-570, 612-655), residual norms of
// ADMMCoordinator._check_convergence (modules/dmpc/admm/admm_coordinator.py:354-435).
//
// All kernels are HBM-bound streaming passes over [rows][T] fp64 trajectories.
// Layout: grid.y = coupling group (alias), grid.x = chunks of ROWS_PER_BLOCK
// participant rows; sums are formed in LDS and added to global with fp64 atomics
// (one atomic per (block, t)), so a group of 16k participants spreads over 64
// workgroups instead of serialising on one CU.
#include <hip/hip_runtime.h>

#include "mpcx.h"

namespace {

constexpr int THREADS = 256;
constexpr int ROWS_PER_BLOCK = 256;
constexpr int MAX_T = 512;

__global__ void __launch_bounds__(THREADS)
k_group_sums(int T, const int* __restrict__ gstart, const double* __restrict__ x,
             const int* __restrict__ active, double* __restrict__ sums) {
  __shared__ double acc[MAX_T + 1];
  const int g = blockIdx.y;
  const int r0 = gstart[g], r1 = gstart[g + 1];
  const int rb = r0 + blockIdx.x * ROWS_PER_BLOCK;
  if (rb >= r1) return;
  const int re = min(rb + ROWS_PER_BLOCK, r1);
  for (int t = threadIdx.x; t <= T; t += THREADS) acc[t] = 0.0;
  __syncthreads();
  const long base = (long)rb * T;
  const int n = (re - rb) * T;
  for (int e = threadIdx.x; e < n; e += THREADS) {
    const int row = rb + e / T;
    if (active && !active[row]) continue;
    atomicAdd(&acc[e % T], x[base + e]);
  }
  for (int row = rb + threadIdx.x; row < re; row += THREADS)
    if (!active || active[row]) atomicAdd(&acc[T], 1.0);
  __syncthreads();
  for (int t = threadIdx.x; t <= T; t += THREADS)
    if (acc[t] != 0.0) atomicAdd(&sums[(long)g * (T + 1) + t], acc[t]);
}

__global__ void k_mean_from_sums(int n_groups, int T, const double* __restrict__ sums,
                                 double* __restrict__ mean, double* __restrict__ dmean) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_groups * T) return;
  const int g = e / T, t = e % T;
  const double cnt = sums[(long)g * (T + 1) + T];
  if (cnt <= 0.0) return;
  const double m = sums[(long)g * (T + 1) + t] / cnt;
  dmean[e] = mean[e] - m;
  mean[e] = m;
}

__global__ void __launch_bounds__(THREADS)
k_consensus_mult(int T, const int* __restrict__ gstart, const double* __restrict__ x,
                 const int* __restrict__ active, const double* __restrict__ mean, double rho,
                 double* __restrict__ lam, double* __restrict__ res) {
  const int g = blockIdx.y;
  const int r0 = gstart[g], r1 = gstart[g + 1];
  const int rb = r0 + blockIdx.x * ROWS_PER_BLOCK;
  if (rb >= r1) return;
  const int re = min(rb + ROWS_PER_BLOCK, r1);
  const long base = (long)rb * T;
  const int n = (re - rb) * T;
  for (int e = threadIdx.x; e < n; e += THREADS) {
    const int row = rb + e / T;
    if (active && !active[row]) { res[base + e] = 0.0; continue; }
    const double r = mean[(long)g * T + e % T] - x[base + e];
    res[base + e] = r;
    lam[base + e] -= rho * r;
  }
}

__global__ void __launch_bounds__(THREADS)
k_exchange_diff(int T, const int* __restrict__ gstart, const double* __restrict__ x,
                const int* __restrict__ active, const double* __restrict__ mean,
                double* __restrict__ diff) {
  const int g = blockIdx.y;
  const int r0 = gstart[g], r1 = gstart[g + 1];
  const int rb = r0 + blockIdx.x * ROWS_PER_BLOCK;
  if (rb >= r1) return;
  const int re = min(rb + ROWS_PER_BLOCK, r1);
  const long base = (long)rb * T;
  const int n = (re - rb) * T;
  for (int e = threadIdx.x; e < n; e += THREADS) {
    const int row = rb + e / T;
    if (active && !active[row]) continue;
    diff[base + e] = x[base + e] - mean[(long)g * T + e % T];
  }
}

__global__ void k_exchange_mult(int n_groups, int T, const double* __restrict__ mean, double rho,
                                double* __restrict__ lam, double* __restrict__ res) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_groups * T) return;
  const double m = mean[e];
  res[e] = m;
  lam[e] += rho * m;
}

__global__ void __launch_bounds__(THREADS)
k_residual_partials(int T, const int* __restrict__ gstart, const double* __restrict__ res,
                    const double* __restrict__ dmean, const double* __restrict__ x,
                    const double* __restrict__ lam, const int* __restrict__ active, double rho,
                    int exchange, double* __restrict__ out) {
  __shared__ double acc[4];
  const int g = blockIdx.y;
  const int r0 = gstart[g], r1 = gstart[g + 1];
  const int rb = r0 + blockIdx.x * ROWS_PER_BLOCK;
  if (rb >= r1) return;
  const int re = min(rb + ROWS_PER_BLOCK, r1);
  if (threadIdx.x < 4) acc[threadIdx.x] = 0.0;
  __syncthreads();
  double s_r = 0.0, s_x = 0.0, s_l = 0.0, s_d = 0.0;
  const long base = (long)rb * T;
  const int n = (re - rb) * T;
  for (int e = threadIdx.x; e < n; e += THREADS) {
    const int row = rb + e / T;
    if (active && !active[row]) continue;
    const double xv = x[base + e];
    s_x += xv * xv;
    if (!exchange) {
      const double r = res[base + e], l = lam[base + e];
      s_r += r * r;
      s_l += l * l;
    }
  }
  if (blockIdx.x == 0) {  // per-group terms counted once
    for (int t = threadIdx.x; t < T; t += THREADS) {
      const double d = rho * dmean[(long)g * T + t];
      s_d += d * d;
      if (exchange) {
        const double r = res[(long)g * T + t], l = lam[(long)g * T + t];
        s_r += r * r;
        s_l += l * l;
      }
    }
  }
  atomicAdd(&acc[0], s_r);
  atomicAdd(&acc[1], s_d);
  atomicAdd(&acc[2], s_x);
  atomicAdd(&acc[3], s_l);
  __syncthreads();
  if (threadIdx.x < 4) atomicAdd(&out[(long)g * 4 + threadIdx.x], acc[threadIdx.x]);
}

__global__ void k_shift(int n_rows, int T, int shift, double* __restrict__ x) {
  // reference: seq[shift:] + seq[-shift:] — the tail keeps the last `shift` values
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n_rows) return;
  double* r = x + (long)row * T;
  for (int t = 0; t < T - shift; ++t) r[t] = r[t + shift];
}

inline dim3 group_grid(int n_groups, const int* /*gstart (device)*/, int max_rows) {
  const int chunks = (max_rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  return dim3(chunks > 0 ? chunks : 1, n_groups, 1);
}

}  // namespace

#define LAUNCH_CHECK()                                        \
  do {                                                        \
    if (hipGetLastError() != hipSuccess) return MPCX_ERR_HIP; \
  } while (0)

extern "C" int mpcx_admm_group_sums(int32_t n_groups, int32_t T, const int32_t* gstart,
                                    int32_t max_group_rows,
                                    const double* locals, const int32_t* active, double* sums,
                                    void* stream) {
  if (n_groups <= 0 || T <= 0 || T > MAX_T || !gstart || !locals || !sums) return MPCX_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int mr = max_group_rows;
  hipLaunchKernelGGL(k_group_sums, group_grid(n_groups, gstart, mr), dim3(THREADS), 0, s, T, gstart,
                     locals, active, sums);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_admm_mean_from_sums(int32_t n_groups, int32_t T, const double* sums,
                                        double* mean, double* delta_mean, void* stream) {
  if (n_groups <= 0 || T <= 0 || !sums || !mean || !delta_mean) return MPCX_ERR_ARG;
  const int n = n_groups * T;
  hipLaunchKernelGGL(k_mean_from_sums, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     n_groups, T, sums, mean, delta_mean);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_admm_consensus_multipliers(int32_t n_groups, int32_t T, const int32_t* gstart,
                                    int32_t max_group_rows,
                                               const double* locals, const int32_t* active,
                                               const double* mean, double rho, double* mult,
                                               double* res, void* stream) {
  if (n_groups <= 0 || T <= 0 || !gstart || !locals || !mean || !mult || !res) return MPCX_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int mr = max_group_rows;
  hipLaunchKernelGGL(k_consensus_mult, group_grid(n_groups, gstart, mr), dim3(THREADS), 0, s, T,
                     gstart, locals, active, mean, rho, mult, res);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_admm_exchange_update(int32_t n_groups, int32_t T, const int32_t* gstart,
                                    int32_t max_group_rows,
                                         const double* locals, const int32_t* active,
                                         const double* mean, double* diff, double* mult,
                                         double* res, double rho, void* stream) {
  if (n_groups <= 0 || T <= 0 || !gstart || !locals || !mean || !diff || !mult || !res)
    return MPCX_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int mr = max_group_rows;
  hipLaunchKernelGGL(k_exchange_diff, group_grid(n_groups, gstart, mr), dim3(THREADS), 0, s, T,
                     gstart, locals, active, mean, diff);
  LAUNCH_CHECK();
  const int n = n_groups * T;
  hipLaunchKernelGGL(k_exchange_mult, dim3((n + 255) / 256), dim3(256), 0, s, n_groups, T, mean,
                     rho, mult, res);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_admm_residual_partials(int32_t n_groups, int32_t T, const int32_t* gstart,
                                    int32_t max_group_rows,
                                           const double* res, const double* dmean,
                                           const double* locals, const double* mult,
                                           const int32_t* active, double rho, int32_t exchange,
                                           double* out, void* stream) {
  if (n_groups <= 0 || T <= 0 || !gstart || !res || !dmean || !locals || !mult || !out)
    return MPCX_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int mr = max_group_rows;
  hipLaunchKernelGGL(k_residual_partials, group_grid(n_groups, gstart, mr), dim3(THREADS), 0, s, T,
                     gstart, res, dmean, locals, mult, active, rho, exchange, out);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_admm_shift(int32_t n_rows, int32_t T, int32_t shift, double* x, void* stream) {
  if (n_rows < 0 || T <= 0 || shift < 0 || shift > T || !x) return MPCX_ERR_ARG;
  if (n_rows == 0 || shift == 0) return MPCX_OK;
  hipLaunchKernelGGL(k_shift, dim3((n_rows + 255) / 256), dim3(256), 0, (hipStream_t)stream, n_rows,
                     T, shift, x);
  LAUNCH_CHECK();
  return MPCX_OK;
}
