// admm_kernels.hip — agent-batched ADMM arithmetic (consensus and exchange) and the
// NLP-vector <-> trajectory moves around it.
//
// Reference semantics: ConsensusVariable / ExchangeVariable
// (agentlib_mpc/data_structures/admm_datatypes.py:202-331), ADMM._set_mean_coupling_values
// and update_lambda (modules/dmpc/admm/admm.py:528-655), the residual norms and stopping
// rule of ADMMCoordinator._check_convergence (modules/dmpc/admm/admm_coordinator.py:354-435).
//
// Layout: local trajectories are rows of X [n_rows][T] (fp64), the participants of one
// coupling alias ("group") are the contiguous rows gstart[g] .. gstart[g+1]-1.
// Every kernel is an HBM-bound streaming pass; the only reductions are per (group, t)
// and use registers -> LDS -> one fp64 atomic per (workgroup, value).
//
// One all-reduce per ADMM iteration: mpcx_admm_moments forms, per (group, t), the
// moments of the locals about the CURRENT mean c (the "old" mean):
//   S1 = sum (x - c), S2 = sum (x - c)^2, SL = sum lam, SL2 = sum lam^2, SLX = sum lam (x - c)
// plus the participant count.  Everything the reference computes from the individual
// rows after the mean is known follows from them exactly (m = c + S1/n):
//   sum (m - x)^2                 = S2 - S1^2/n                      (primal residual)
//   sum (lam + rho (x - m))^2     = SL2 + 2 rho (SLX - (m - c) SL) + rho^2 (S2 - S1^2/n)
//   sum x^2                       = S2 + 2 c S1 + n c^2
// so groups whose participants live on several GPUs need only their moments summed
// across ranks (RCCL all-reduce) before mpcx_admm_finalize.
//
// Blocks: the groups are partitioned into independent consensus blocks (one reference
// ADMMCoordinator each, e.g. the 4-room + air-handler blocks of a scaled C2 fleet).  The
// residual totals are kept per block ([n_blocks][MPCX_ADMM_TOTALS]), every group may carry
// its own penalty rho_g (penalty variation per coordinator), and groups whose block has
// converged (active_g == 0) are frozen: no mean, multiplier or diff update.
#include <hip/hip_runtime.h>

#include "mpcx.h"

namespace {

constexpr int THREADS = 256;
constexpr int ROWS_PER_BLOCK = 256;
constexpr int NMOM = 5;            // S1, S2, SL, SL2, SLX
constexpr int WAVE = 64;

// moments buffer: [global groups][totals: n_blocks x MPCX_ADMM_TOTALS][local groups]
__device__ __forceinline__ long mom_offset(int g, int g_global, int T, int n_tot) {
  const long S = (long)NMOM * T + 1;
  return (long)g * S + (g >= g_global ? n_tot : 0);
}
__device__ __forceinline__ bool g_active(const int* active_g, int g) { return active_g == nullptr || active_g[g] != 0; }
__device__ __forceinline__ double g_rho(const double* rho_g, double rho, int g) { return rho_g ? rho_g[g] : rho; }

// --- NLP vector <-> trajectory rows ---------------------------------------------------
__global__ void k_gather_rows(int n, int T, const double* __restrict__ src, long ld,
                              const int* __restrict__ cols, double* __restrict__ dst,
                              const int* __restrict__ dst_rows) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * T) return;
  const int a = (int)(e / T), t = (int)(e % T);
  dst[(long)dst_rows[a] * T + t] = src[(long)a * ld + cols[t]];
}

__global__ void k_scatter_rows(int n, int T, const double* __restrict__ src,
                               const int* __restrict__ src_rows, double* __restrict__ dst, long ld,
                               const int* __restrict__ cols) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * T) return;
  const int a = (int)(e / T), t = (int)(e % T);
  const long r = src_rows ? src_rows[a] : a;
  dst[(long)a * ld + cols[t]] = src[r * T + t];
}

// Several row moves in one launch (C ABI v12): blockIdx.y selects a descriptor of MPCX_MOVE_DESC
// int64 words in device memory.  Scatter descriptor: (src, src_rows or 0, cols, T) into the common
// destination; gather descriptor: (dst, dst_rows, cols, T) from the common source.
__global__ void k_scatter_rows_multi(int n, const long long* __restrict__ desc, double* __restrict__ dst,
                                     long ld) {
  const long long* d = desc + (long)blockIdx.y * MPCX_MOVE_DESC;
  const int T = (int)d[3];
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * T) return;
  const double* src = (const double*)d[0];
  const int* rows = (const int*)d[1];
  const int* cols = (const int*)d[2];
  const int a = (int)(e / T), t = (int)(e % T);
  const long r = rows ? rows[a] : a;
  dst[(long)a * ld + cols[t]] = src[r * T + t];
}

__global__ void k_gather_rows_multi(int n, const long long* __restrict__ desc, const double* __restrict__ src,
                                    long ld) {
  const long long* d = desc + (long)blockIdx.y * MPCX_MOVE_DESC;
  const int T = (int)d[3];
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * T) return;
  double* dst = (double*)d[0];
  const int* rows = (const int*)d[1];
  const int* cols = (const int*)d[2];
  const int a = (int)(e / T), t = (int)(e % T);
  dst[(long)rows[a] * T + t] = src[(long)a * ld + cols[t]];
}

__global__ void k_fill_column(int n, double* __restrict__ dst, long ld, int col, double v) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a < n) dst[(long)a * ld + col] = v;
}

// --- moments -----------------------------------------------------------------------------
// grid (n_groups, row chunks). Thread (r, tc): column t0+tc, rows rb+r, rb+r+R, ...
__global__ void __launch_bounds__(THREADS)
k_moments(int g_global, int n_tot, int T, const int* __restrict__ gstart, const double* __restrict__ x,
          const double* __restrict__ lam, const double* __restrict__ center,
          const int* __restrict__ row_on, double* __restrict__ out) {
  __shared__ double part[THREADS * NMOM];
  const int g = blockIdx.x;
  const int r0 = gstart[g], r1 = gstart[g + 1];
  const int rb = r0 + blockIdx.y * ROWS_PER_BLOCK;
  if (rb >= r1) return;
  const int re = min(rb + ROWS_PER_BLOCK, r1);
  double* o = out + mom_offset(g, g_global, T, n_tot);
  const int cpp = T < THREADS ? T : THREADS;  // columns per pass
  const int R = THREADS / cpp;                // row lanes
  const int r = threadIdx.x / cpp, tc = threadIdx.x % cpp;
  for (int t0 = 0; t0 < T; t0 += cpp) {
    const int t = t0 + tc;
    double s1 = 0.0, s2 = 0.0, sl = 0.0, sl2 = 0.0, slx = 0.0;
    if (r < R && t < T) {
      const double c = center[(long)g * T + t];
      for (int row = rb + r; row < re; row += R) {
        if (row_on && !row_on[row]) continue;  // not participating this round
        const double d = x[(long)row * T + t] - c;
        s1 += d;
        s2 += d * d;
        if (lam) {
          const double l = lam[(long)row * T + t];
          sl += l;
          sl2 += l * l;
          slx += l * d;
        }
      }
    }
    double* p = part + threadIdx.x * NMOM;
    p[0] = s1; p[1] = s2; p[2] = sl; p[3] = sl2; p[4] = slx;
    __syncthreads();
    if (r == 0 && t < T) {
      for (int q = 1; q < R; ++q) {
        const double* pq = part + (q * cpp + tc) * NMOM;
        s1 += pq[0]; s2 += pq[1]; sl += pq[2]; sl2 += pq[3]; slx += pq[4];
      }
      atomicAdd(&o[0 * T + t], s1);
      atomicAdd(&o[1 * T + t], s2);
      if (lam) {
        atomicAdd(&o[2 * T + t], sl);
        atomicAdd(&o[3 * T + t], sl2);
        atomicAdd(&o[4 * T + t], slx);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int cnt = re - rb;
    if (row_on)
      for (int row = rb; row < re; ++row) cnt -= row_on[row] ? 0 : 1;
    atomicAdd(&o[NMOM * T], (double)cnt);
  }
}

// --- finalize: one wavefront per group ------------------------------------------------
__global__ void __launch_bounds__(WAVE)
k_finalize(int g0, int g1, int g_global, int n_tot, int T, const double* __restrict__ mom,
           const int* __restrict__ exchange, const double* __restrict__ gmult, double rho_s,
           const double* __restrict__ rho_g, const int* __restrict__ active_g,
           const int* __restrict__ block_g, double* __restrict__ mean, double* __restrict__ dmean,
           double* __restrict__ totals_all) {
  const int g = g0 + blockIdx.x;
  if (g >= g1 || !g_active(active_g, g)) return;
  const double rho = g_rho(rho_g, rho_s, g);
  double* totals = totals_all + (block_g ? (long)block_g[g] * MPCX_ADMM_TOTALS : 0);
  const double* o = mom + mom_offset(g, g_global, T, n_tot);
  const double n = o[NMOM * T];
  const bool ex = exchange && exchange[g];
  double prim = 0.0, dual = 0.0, xs = 0.0, ms = 0.0, ls = 0.0;
  if (n > 0.0) {
    for (int t = threadIdx.x; t < T; t += WAVE) {
      const double c = mean[(long)g * T + t];
      const double s1 = o[t], s2 = o[T + t];
      const double dm = s1 / n;                 // m - c
      const double m = c + dm;
      const double var = fmax(s2 - s1 * dm, 0.0);  // sum (x - m)^2
      mean[(long)g * T + t] = m;
      dmean[(long)g * T + t] = c - m;           // delta_mean = old - new
      const double dd = rho * (c - m);
      dual += dd * dd;
      xs += s2 + 2.0 * c * s1 + n * c * c;
      ms += m * m;
      if (ex) {
        prim += m * m;                          // exchange primal residual = mean
        const double l = gmult[(long)g * T + t] + rho * m;
        ls += l * l;
      } else {
        prim += var;
        const double sl = o[2 * T + t], sl2 = o[3 * T + t], slx = o[4 * T + t];
        ls += sl2 + 2.0 * rho * (slx - dm * sl) + rho * rho * var;
      }
    }
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    prim += __shfl_xor(prim, s, WAVE);
    dual += __shfl_xor(dual, s, WAVE);
    xs += __shfl_xor(xs, s, WAVE);
    ms += __shfl_xor(ms, s, WAVE);
    ls += __shfl_xor(ls, s, WAVE);
  }
  if (threadIdx.x == 0 && n > 0.0) {
    atomicAdd(&totals[0], prim);
    atomicAdd(&totals[1], dual);
    atomicAdd(&totals[2], xs);
    atomicAdd(&totals[3], ms);
    atomicAdd(&totals[4], ls);
    atomicAdd(&totals[5], n);                   // trajectories (flat_locals entries)
    atomicAdd(&totals[6], ex ? (double)T : n);  // flat_multipliers entries (reference quirk)
    atomicAdd(&totals[7], 1.0);                 // groups with participants
  }
}

// --- multiplier / diff updates ---------------------------------------------------------
__global__ void __launch_bounds__(THREADS)
k_consensus_mult(int T, const int* __restrict__ gstart, const double* __restrict__ x,
                 const double* __restrict__ mean, double rho_s, const double* __restrict__ rho_g,
                 const int* __restrict__ active_g, const int* __restrict__ row_on, double* __restrict__ lam,
                 double* __restrict__ res) {
  const int g = blockIdx.x;
  if (!g_active(active_g, g)) return;
  const double rho = g_rho(rho_g, rho_s, g);
  const int r0 = gstart[g], r1 = gstart[g + 1];
  const int rb = r0 + blockIdx.y * ROWS_PER_BLOCK;
  if (rb >= r1) return;
  const int re = min(rb + ROWS_PER_BLOCK, r1);
  const long base = (long)rb * T;
  const int n = (re - rb) * T;
  for (int e = threadIdx.x; e < n; e += THREADS) {
    if (row_on && !row_on[rb + e / T]) continue;  // not participating: multiplier kept
    const double r = mean[(long)g * T + e % T] - x[base + e];
    if (res) res[base + e] = r;
    lam[base + e] -= rho * r;
  }
}

__global__ void __launch_bounds__(THREADS)
k_exchange_diff(int T, const int* __restrict__ gstart, const double* __restrict__ x,
                const double* __restrict__ mean, const int* __restrict__ active_g,
                const int* __restrict__ row_on, double* __restrict__ diff) {
  const int g = blockIdx.x;
  if (!g_active(active_g, g)) return;
  const int r0 = gstart[g], r1 = gstart[g + 1];
  const int rb = r0 + blockIdx.y * ROWS_PER_BLOCK;
  if (rb >= r1) return;
  const int re = min(rb + ROWS_PER_BLOCK, r1);
  const long base = (long)rb * T;
  const int n = (re - rb) * T;
  for (int e = threadIdx.x; e < n; e += THREADS)
    if (!row_on || row_on[rb + e / T]) diff[base + e] = x[base + e] - mean[(long)g * T + e % T];
}

__global__ void k_exchange_mult(int n_groups, int T, const double* __restrict__ mean, double rho_s,
                                const double* __restrict__ rho_g, const int* __restrict__ active_g,
                                double* __restrict__ lam) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_groups * T) return;
  const int g = e / T;
  if (!g_active(active_g, g)) return;
  lam[e] += g_rho(rho_g, rho_s, g) * mean[e];
}

__global__ void k_shift(int n_rows, int T, int shift, double* __restrict__ x) {
  // reference: seq[shift:] + seq[-shift:] — the tail keeps the last `shift` values
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n_rows) return;
  double* r = x + (long)row * T;
  for (int t = 0; t < T - shift; ++t) r[t] = r[t + shift];
}

inline dim3 group_grid(int n_groups, int max_rows) {
  const int chunks = (max_rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  return dim3(n_groups, chunks > 0 ? chunks : 1, 1);
}

inline unsigned blocks_for(long n, int threads) { return (unsigned)((n + threads - 1) / threads); }

}  // namespace

#define LAUNCH_CHECK()                                        \
  do {                                                        \
    if (hipGetLastError() != hipSuccess) return MPCX_ERR_HIP; \
  } while (0)

extern "C" int mpcx_gather_rows(int32_t n_agents, int32_t T, const double* src, int64_t src_ld,
                                const int32_t* cols, double* dst, const int32_t* dst_rows,
                                void* stream) {
  if (n_agents < 0 || T <= 0 || src_ld <= 0 || !src || !cols || !dst || !dst_rows) return MPCX_ERR_ARG;
  if (n_agents == 0) return MPCX_OK;
  const long n = (long)n_agents * T;
  hipLaunchKernelGGL(k_gather_rows, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     n_agents, T, src, (long)src_ld, cols, dst, dst_rows);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_scatter_rows(int32_t n_agents, int32_t T, const double* src,
                                 const int32_t* src_rows, double* dst, int64_t dst_ld,
                                 const int32_t* cols, void* stream) {
  if (n_agents < 0 || T <= 0 || dst_ld <= 0 || !src || !dst || !cols) return MPCX_ERR_ARG;
  if (n_agents == 0) return MPCX_OK;
  const long n = (long)n_agents * T;
  hipLaunchKernelGGL(k_scatter_rows, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     n_agents, T, src, src_rows, dst, (long)dst_ld, cols);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_scatter_rows_multi(int32_t n_agents, int32_t n_desc, const int64_t* desc, int32_t max_T,
                                       double* dst, int64_t dst_ld, void* stream) {
  if (n_agents < 0 || n_desc < 0 || max_T <= 0 || dst_ld <= 0 || !dst || (n_desc > 0 && !desc)) return MPCX_ERR_ARG;
  if (n_agents == 0 || n_desc == 0) return MPCX_OK;
  const long n = (long)n_agents * max_T;
  hipLaunchKernelGGL(k_scatter_rows_multi, dim3(blocks_for(n, 256), n_desc), dim3(256), 0, (hipStream_t)stream,
                     n_agents, (const long long*)desc, dst, (long)dst_ld);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_gather_rows_multi(int32_t n_agents, int32_t n_desc, const int64_t* desc, int32_t max_T,
                                      const double* src, int64_t src_ld, void* stream) {
  if (n_agents < 0 || n_desc < 0 || max_T <= 0 || src_ld <= 0 || !src || (n_desc > 0 && !desc)) return MPCX_ERR_ARG;
  if (n_agents == 0 || n_desc == 0) return MPCX_OK;
  const long n = (long)n_agents * max_T;
  hipLaunchKernelGGL(k_gather_rows_multi, dim3(blocks_for(n, 256), n_desc), dim3(256), 0, (hipStream_t)stream,
                     n_agents, (const long long*)desc, src, (long)src_ld);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_fill_column(int32_t n_agents, double* dst, int64_t dst_ld, int32_t col,
                                double value, void* stream) {
  if (n_agents < 0 || dst_ld <= 0 || col < 0 || col >= dst_ld || !dst) return MPCX_ERR_ARG;
  if (n_agents == 0) return MPCX_OK;
  hipLaunchKernelGGL(k_fill_column, dim3(blocks_for(n_agents, 256)), dim3(256), 0,
                     (hipStream_t)stream, n_agents, dst, (long)dst_ld, col, value);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int64_t mpcx_admm_moments_size(int32_t n_groups, int32_t n_blocks, int32_t T) {
  if (n_groups < 0 || n_blocks < 1 || T <= 0) return MPCX_ERR_ARG;
  return (int64_t)n_groups * (NMOM * (int64_t)T + 1) + (int64_t)MPCX_ADMM_TOTALS * n_blocks;
}

// Length of the all-reduced range (C ABI v10): the control doubles right before the moments
// buffer (the coordinated loop's count of blocks still active), the global groups' moments,
// then the totals of the blocks that span ranks (numbered first, identically on every rank;
// the rank-local blocks' totals follow them and stay local).
extern "C" int64_t mpcx_admm_reduce_count(int32_t n_global, int32_t n_global_blocks, int32_t T) {
  if (n_global < 0 || n_global_blocks < 0 || T <= 0) return MPCX_ERR_ARG;
  return (int64_t)MPCX_ADMM_CONTROL + (int64_t)n_global * (NMOM * (int64_t)T + 1) +
         (int64_t)MPCX_ADMM_TOTALS * n_global_blocks;
}

extern "C" int mpcx_admm_moments_masked(int32_t n_groups, int32_t n_global, int32_t n_blocks, int32_t T,
                                        const int32_t* gstart, int32_t max_group_rows,
                                        const double* locals, const double* multipliers,
                                        const double* center, const int32_t* row_on, double* out,
                                        void* stream) {
  if (n_groups <= 0 || n_global < 0 || n_global > n_groups || n_blocks < 1 || T <= 0 ||
      max_group_rows < 0 || !gstart || !locals || !center || !out)
    return MPCX_ERR_ARG;
  if (max_group_rows == 0) return MPCX_OK;
  hipLaunchKernelGGL(k_moments, group_grid(n_groups, max_group_rows), dim3(THREADS), 0,
                     (hipStream_t)stream, n_global, MPCX_ADMM_TOTALS * n_blocks, T, gstart, locals,
                     multipliers, center, row_on, out);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_admm_moments(int32_t n_groups, int32_t n_global, int32_t n_blocks, int32_t T,
                                 const int32_t* gstart, int32_t max_group_rows,
                                 const double* locals, const double* multipliers,
                                 const double* center, double* out, void* stream) {
  return mpcx_admm_moments_masked(n_groups, n_global, n_blocks, T, gstart, max_group_rows, locals,
                                  multipliers, center, nullptr, out, stream);
}

extern "C" int mpcx_admm_finalize(int32_t g_begin, int32_t g_end, int32_t n_global, int32_t n_blocks,
                                  int32_t T, const double* moments, const int32_t* exchange,
                                  const double* group_multipliers, double rho, const double* rho_g,
                                  const int32_t* active_g, const int32_t* block_g, double* mean,
                                  double* delta_mean, double* totals, void* stream) {
  if (g_begin < 0 || g_end < g_begin || n_global < 0 || n_blocks < 1 || T <= 0 || !moments ||
      !mean || !delta_mean || !totals)
    return MPCX_ERR_ARG;
  if (exchange && !group_multipliers) return MPCX_ERR_ARG;
  if (n_blocks > 1 && !block_g) return MPCX_ERR_ARG;
  if (g_end == g_begin) return MPCX_OK;
  hipLaunchKernelGGL(k_finalize, dim3(g_end - g_begin), dim3(WAVE), 0, (hipStream_t)stream, g_begin,
                     g_end, n_global, MPCX_ADMM_TOTALS * n_blocks, T, moments, exchange,
                     group_multipliers, rho, rho_g, active_g, block_g, mean, delta_mean, totals);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_admm_consensus_multipliers_masked(int32_t n_groups, int32_t T, const int32_t* gstart,
                                                      int32_t max_group_rows, const double* locals,
                                                      const double* mean, double rho, const double* rho_g,
                                                      const int32_t* active_g, const int32_t* row_on,
                                                      double* mult, double* res, void* stream) {
  if (n_groups <= 0 || T <= 0 || max_group_rows < 0 || !gstart || !locals || !mean || !mult)
    return MPCX_ERR_ARG;
  if (max_group_rows == 0) return MPCX_OK;
  hipLaunchKernelGGL(k_consensus_mult, group_grid(n_groups, max_group_rows), dim3(THREADS), 0,
                     (hipStream_t)stream, T, gstart, locals, mean, rho, rho_g, active_g, row_on, mult, res);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_admm_consensus_multipliers(int32_t n_groups, int32_t T, const int32_t* gstart,
                                               int32_t max_group_rows, const double* locals,
                                               const double* mean, double rho, const double* rho_g,
                                               const int32_t* active_g, double* mult, double* res,
                                               void* stream) {
  return mpcx_admm_consensus_multipliers_masked(n_groups, T, gstart, max_group_rows, locals, mean, rho,
                                                rho_g, active_g, nullptr, mult, res, stream);
}

extern "C" int mpcx_admm_exchange_update_masked(int32_t n_groups, int32_t T, const int32_t* gstart,
                                                int32_t max_group_rows, const double* locals,
                                                const double* mean, double* diff, double* mult,
                                                int32_t update_multiplier, double rho, const double* rho_g,
                                                const int32_t* active_g, const int32_t* row_on,
                                                void* stream) {
  if (n_groups <= 0 || T <= 0 || max_group_rows < 0 || !gstart || !locals || !mean || !diff)
    return MPCX_ERR_ARG;
  if (update_multiplier && !mult) return MPCX_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (max_group_rows > 0) {
    hipLaunchKernelGGL(k_exchange_diff, group_grid(n_groups, max_group_rows), dim3(THREADS), 0, s,
                       T, gstart, locals, mean, active_g, row_on, diff);
    LAUNCH_CHECK();
  }
  if (update_multiplier) {
    const int n = n_groups * T;
    hipLaunchKernelGGL(k_exchange_mult, dim3(blocks_for(n, 256)), dim3(256), 0, s, n_groups, T,
                       mean, rho, rho_g, active_g, mult);
    LAUNCH_CHECK();
  }
  return MPCX_OK;
}

extern "C" int mpcx_admm_exchange_update(int32_t n_groups, int32_t T, const int32_t* gstart,
                                         int32_t max_group_rows, const double* locals,
                                         const double* mean, double* diff, double* mult,
                                         int32_t update_multiplier, double rho, const double* rho_g,
                                         const int32_t* active_g, void* stream) {
  return mpcx_admm_exchange_update_masked(n_groups, T, gstart, max_group_rows, locals, mean, diff, mult,
                                          update_multiplier, rho, rho_g, active_g, nullptr, stream);
}

extern "C" int mpcx_admm_shift(int32_t n_rows, int32_t T, int32_t shift, double* x, void* stream) {
  if (n_rows < 0 || T <= 0 || shift < 0 || shift > T || !x) return MPCX_ERR_ARG;
  if (n_rows == 0 || shift == 0) return MPCX_OK;
  hipLaunchKernelGGL(k_shift, dim3(blocks_for(n_rows, 256)), dim3(256), 0, (hipStream_t)stream,
                     n_rows, T, shift, x);
  LAUNCH_CHECK();
  return MPCX_OK;
}

// --- the coordinators' stopping test on the device ------------------------------------------
// One thread per block (one reference ADMMCoordinator each): ADMMCoordinator._check_convergence
// (admm_coordinator.py:354-435) on the block's residual totals of this iteration, the penalty
// variation (:467-479, recorded after it, :396-402), and the loop's freeze of a converged block
// (:288-304) -- so that a fleet iteration needs no host round trip: the host reads the number
// of active blocks only every few iterations and the records once per round.
namespace {
__global__ void k_block_stop(int nb, int it, const double* __restrict__ totals, int use_rel, double abs_tol,
                             double rel_tol, double primal_tol, double dual_tol, double thr, double fac,
                             double* __restrict__ rho_b, int* __restrict__ active_b, int* __restrict__ iters_b,
                             double* __restrict__ record, int* __restrict__ n_active, long long* __restrict__ clock) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b == 0 && clock) clock[it] = (long long)wall_clock64();
  if (b >= nb) return;
  if (it == 0) {  // the round's start: stamp the clock, count the blocks that will iterate
    if (n_active && active_b && active_b[b] != 0) atomicAdd(n_active, 1);
    return;
  }
  const double* t = totals + (long)b * MPCX_ADMM_TOTALS;
  const double prim = sqrt(fmax(t[0], 0.0)), dual = sqrt(fmax(t[1], 0.0));
  bool conv;
  if (use_rel) {
    const double scale_p = fmax(sqrt(fmax(t[2], 0.0)), sqrt(fmax(t[3], 0.0)));
    const double eps_pri = sqrt(t[6]) * abs_tol + rel_tol * scale_p;
    const double eps_dual = sqrt(t[5]) * abs_tol + rel_tol * sqrt(fmax(t[4], 0.0));
    conv = prim < eps_pri && dual < eps_dual;
  } else {
    conv = prim < primal_tol && dual < dual_tol;
  }
  const bool act = active_b[b] != 0;
  double rho = rho_b[b];
  if (thr > 1.0 && act) {
    if (prim > thr * dual) rho = rho * fac;
    else if (dual > thr * prim) rho = rho / fac;
    rho_b[b] = rho;
  }
  double* r = record + ((long)(it - 1) * nb + b) * 4;
  r[0] = prim; r[1] = dual; r[2] = rho; r[3] = act ? 1.0 : 0.0;
  const bool still = act && !conv;
  if (act && conv) { active_b[b] = 0; iters_b[b] = it; }
  if (n_active && still) atomicAdd(n_active + it, 1);
}

// the count of blocks still active as a double in the caller's control slot (the first double
// of the all-reduced range, C ABI v10): one plain store after k_block_stop's atomics have landed
__global__ void k_control_store(const int* __restrict__ n_active, double* __restrict__ control) {
  if (threadIdx.x == 0) control[0] = (double)n_active[0];
}

__global__ void k_block_expand(int n, const int* __restrict__ idx, const int* __restrict__ active_b,
                               const double* __restrict__ rho_b, const int* __restrict__ part,
                               int* __restrict__ out_active, double* __restrict__ out_rho) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int b = idx[i];
  if (out_active) out_active[i] = (active_b[b] != 0 && (part == nullptr || part[i] != 0)) ? 1 : 0;
  if (out_rho) out_rho[i] = rho_b[b];
}

// compaction of an active mask into an agent map (one workgroup, chunks of THREADS entries:
// ballot + popcount prefix per wave, wave offsets through LDS, a running base across chunks)
__global__ void __launch_bounds__(THREADS) k_active_map(int n, const int* __restrict__ active,
                                                        int* __restrict__ map, int* __restrict__ count) {
  __shared__ int wave_cnt[THREADS / WAVE];
  __shared__ int base_s;
  const int t = threadIdx.x, lane = t & (WAVE - 1), w = t / WAVE;
  if (t == 0) base_s = 0;
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += THREADS) {
    const int i = c0 + t;
    const bool on = i < n && active[i] != 0;
    const unsigned long long bal = __ballot(on);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wave_cnt[w] = __popcll(bal);
    __syncthreads();
    int off = base_s;
    for (int q = 0; q < w; ++q) off += wave_cnt[q];
    if (on) map[off + before] = i;
    __syncthreads();
    if (t == 0) {
      int tot = 0;
      for (int q = 0; q < THREADS / WAVE; ++q) tot += wave_cnt[q];
      base_s += tot;
    }
    __syncthreads();
  }
  const int m = base_s;
  for (int i = m + t; i < n; i += THREADS) map[i] = -1;
  if (t == 0) count[0] = m;
}

// a class's batched solve, counted for the fleet's bookkeeping: counts[0] += agents whose status
// is Solve_Succeeded / Solved_To_Acceptable_Level, counts[1] += their restoration-phase calls;
// agents with active[i] == 0 (frozen blocks, not solved) are skipped.  One atomic per wave.
__global__ void k_stats_count(int n, const mpcx_stats* __restrict__ st, const int* __restrict__ active,
                              unsigned long long* __restrict__ counts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int ok = 0, fb = 0;
  if (i < n && (active == nullptr || active[i] != 0)) {
    const int s = st[i].status;
    ok = (s == 0 || s == 1) ? 1 : 0;
    fb = st[i].n_restorations;
  }
#pragma unroll
  for (int o = WAVE / 2; o > 0; o >>= 1) {
    ok += __shfl_xor(ok, o, WAVE);
    fb += __shfl_xor(fb, o, WAVE);
  }
  if ((threadIdx.x & (WAVE - 1)) == 0) {
    if (ok) atomicAdd(counts, (unsigned long long)ok);
    if (fb) atomicAdd(counts + 1, (unsigned long long)fb);
  }
}
// several classes' block expansions / stats counts in one launch (C ABI v15): blockIdx.y selects
// the descriptor (include/mpcx.h)
__global__ void k_block_expand_multi(const long long* __restrict__ desc, const int* __restrict__ active_b,
                                     const double* __restrict__ rho_b) {
  const long long* d = desc + (long)blockIdx.y * MPCX_EXPAND_DESC;
  const int n = (int)d[0];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int* idx = (const int*)d[1];
  const int* part = (const int*)d[2];
  int* out_active = (int*)d[3];
  double* out_rho = (double*)d[4];
  const int b = idx[i];
  if (out_active) out_active[i] = (active_b[b] != 0 && (part == nullptr || part[i] != 0)) ? 1 : 0;
  if (out_rho) out_rho[i] = rho_b[b];
}

__global__ void k_stats_count_multi(const long long* __restrict__ desc, unsigned long long* __restrict__ counts) {
  const long long* d = desc + (long)blockIdx.y * MPCX_STATS_DESC;
  const int n = (int)d[0];
  const mpcx_stats* st = (const mpcx_stats*)d[1];
  const int* active = (const int*)d[2];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int ok = 0, fb = 0;
  if (i < n && (active == nullptr || active[i] != 0)) {
    const int s = st[i].status;
    ok = (s == 0 || s == 1) ? 1 : 0;
    fb = st[i].n_restorations;
  }
#pragma unroll
  for (int o = WAVE / 2; o > 0; o >>= 1) {
    ok += __shfl_xor(ok, o, WAVE);
    fb += __shfl_xor(fb, o, WAVE);
  }
  if ((threadIdx.x & (WAVE - 1)) == 0) {
    if (ok) atomicAdd(counts, (unsigned long long)ok);
    if (fb) atomicAdd(counts + 1, (unsigned long long)fb);
  }
}
}  // namespace

extern "C" int mpcx_admm_block_expand_multi(int32_t n_desc, const int64_t* desc, int32_t max_n,
                                            const int32_t* active_b, const double* rho_b, void* stream) {
  if (n_desc < 0 || max_n < 0 || (n_desc > 0 && (!desc || !active_b))) return MPCX_ERR_ARG;
  if (n_desc == 0 || max_n == 0) return MPCX_OK;
  hipLaunchKernelGGL(k_block_expand_multi, dim3(blocks_for(max_n, 256), n_desc), dim3(256), 0, (hipStream_t)stream,
                     (const long long*)desc, active_b, rho_b);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_stats_count_multi(int32_t n_desc, const int64_t* desc, int32_t max_n, int64_t* counts,
                                      void* stream) {
  if (n_desc < 0 || max_n < 0 || !counts || (n_desc > 0 && !desc)) return MPCX_ERR_ARG;
  if (n_desc == 0 || max_n == 0) return MPCX_OK;
  hipLaunchKernelGGL(k_stats_count_multi, dim3(blocks_for(max_n, 256), n_desc), dim3(256), 0, (hipStream_t)stream,
                     (const long long*)desc, (unsigned long long*)counts);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_stats_count(int32_t n, const mpcx_stats* stats, const int32_t* active, int64_t* counts,
                                void* stream) {
  if (n < 0 || (n > 0 && (!stats || !counts))) return MPCX_ERR_ARG;
  if (n == 0) return MPCX_OK;
  hipLaunchKernelGGL(k_stats_count, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, stats, active,
                     (unsigned long long*)counts);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_active_map(int32_t n, const int32_t* active, int32_t* map, int32_t* count, void* stream) {
  if (n < 0 || (n > 0 && (!active || !map)) || !count) return MPCX_ERR_ARG;
  hipLaunchKernelGGL(k_active_map, dim3(1), dim3(THREADS), 0, (hipStream_t)stream, n, active, map, count);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int mpcx_admm_block_stop(int32_t n_blocks, int32_t it, const double* totals, int32_t use_relative,
                                    double abs_tol, double rel_tol, double primal_tol, double dual_tol,
                                    double change_threshold, double change_factor, double* rho_b,
                                    int32_t* active_b, int32_t* iters_b, double* record, int32_t* n_active,
                                    int64_t* clock, double* control, void* stream) {
  if (n_blocks < 1 || it < 0 || (it > 0 && (!totals || !rho_b || !active_b || !iters_b || !record)))
    return MPCX_ERR_ARG;
  if (control && !n_active) return MPCX_ERR_ARG;
  hipLaunchKernelGGL(k_block_stop, dim3(blocks_for(n_blocks, 256)), dim3(256), 0, (hipStream_t)stream,
                     n_blocks, it, totals, use_relative, abs_tol, rel_tol, primal_tol, dual_tol, change_threshold,
                     change_factor, rho_b, active_b, iters_b, record, n_active, (long long*)clock);
  LAUNCH_CHECK();
  if (control) {
    hipLaunchKernelGGL(k_control_store, dim3(1), dim3(WAVE), 0, (hipStream_t)stream, n_active + it, control);
    LAUNCH_CHECK();
  }
  return MPCX_OK;
}

extern "C" int mpcx_admm_block_expand(int32_t n, const int32_t* idx, const int32_t* active_b, const double* rho_b,
                                      const int32_t* part, int32_t* out_active, double* out_rho, void* stream) {
  if (n < 0 || (n > 0 && !idx) || (out_active && !active_b) || (out_rho && !rho_b)) return MPCX_ERR_ARG;
  if (n == 0 || (!out_active && !out_rho)) return MPCX_OK;
  hipLaunchKernelGGL(k_block_expand, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, idx,
                     active_b, rho_b, part, out_active, out_rho);
  LAUNCH_CHECK();
  return MPCX_OK;
}

extern "C" int64_t mpcx_device_clock_khz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return MPCX_ERR_HIP;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return MPCX_ERR_HIP;
  return khz;
}
