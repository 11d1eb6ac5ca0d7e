// mpcx_ipm.hip — batched primal-dual interior point solver for stage-structured NLPs.
//
// Included at the end of every generated model source (runtime/codegen.py), which
// defines MPCX_N/NX/NV/NG/NPS/NPG/TS and the four gen_stage_* device functions.
//
// What it replaces: the IPOPT solve behind ca.nlpsol (reference
// agentlib_mpc/data_structures/casadi_utils.py:191-217; called at
// optimization_backends/casadi_/core/discretization.py:203).  The algorithm is
// IPOPT's (barrier + slacks, monotone mu, inertia-corrected Newton steps,
// fraction-to-boundary, filter line search, gradient scaling, bound relaxation,
// least-squares multiplier init) and follows the oracle restatement
// oracle/ipm.py step for step.  What differs is the linear algebra: permuted to
// [stage interiors | states], the KKT matrix of a stage-structured NLP has a
// block-diagonal interior part.  Every stage's interior (controls, collocation
// states, outputs, constraint multipliers) is Bunch-Kaufman factored in LDS in
// parallel with the other stages, bordered by the two state blocks it touches
// and by the right-hand side; the local Schur complements on the states form a
// block-tridiagonal chain of nx x nx pivots, the only sequential part.
// Inertia = interior inertias + chain inertia (Haynsworth), exactly what IPOPT
// reads from MUMPS.  A stage whose interior is singular sends the agent to the
// sequential block chain (Riccati through the state columns) instead.
//
// Mapping: one agent per workgroup of one wavefront (64 lanes).  Lanes own
// variables/constraints (i = lane + 64*slot) for the vector phases, stages for
// the generated evaluations, and lane groups of G own stages during the
// factorisation.  The iterate lives in an HBM workspace slab; everything a
// phase hands to lanes of another mapping goes through LDS where it fits
// (parameters, trial point, step, factors), otherwise through the slab plus a
// workgroup barrier.  Phases issue all their global loads before the first
// dependent use: the kernel is latency-bound, not flop-bound.
#include <hip/hip_runtime.h>
#include <math.h>
#include "mpcx.h"
#include "mpcx_internal.h"

namespace mpcx_kernel {

constexpr int N = MPCX_N;
constexpr int NX = MPCX_NX;
constexpr int NV = MPCX_NV;
constexpr int NG = MPCX_NG;
constexpr int NPS = MPCX_NPS;
constexpr int NPG = MPCX_NPG;
constexpr int NL = 2 * NX + NV;    // stage-local vector [X0, V, X1]
constexpr int NP = NV + NX;        // primal unknowns per KKT block [V, X1]
constexpr int NB = NP + NG;        // KKT block size
constexpr int NW = NX + N * NP;    // NLP variables (reference order)
constexpr int M = N * NG;          // NLP constraints
constexpr int MM = M > 0 ? M : 1;
constexpr int NPAR = NPG + N * NPS;
constexpr int LDB = (NB % 2 == 0) ? NB + 1 : NB;
constexpr int WAVE = 64;
constexpr int VS = (NW + WAVE - 1) / WAVE;  // variable slots per lane
constexpr int CS = (M + WAVE - 1) / WAVE;   // constraint slots per lane
// The filter (IPOPT Filter: entries a new one dominates are removed on insertion, AddEntry; the
// list is unbounded).  Its newest MAXF entries live in LDS, one per lane for the filter test; older
// ones move, in insertion order, to a spill list in the agent's HBM workspace (FSPILL entries,
// scanned only while it holds any -- no benchmark case ever fills the LDS part).  Together
// MAXF + FSPILL = 1024 entries, the cap shared with oracle/ipm.py (max_filter) and
// oracle/c/ipm_oracle.c; an insertion into a full filter drops the oldest entry (counted).
// MPCX_MAXF / MPCX_FSPILL: smaller parts for the parity test builds (tests/test_gpu_ipm.py).
// r06: 48 in LDS (was 64): the 256 bytes pay for the per-lane element-class word (ecls) so that no
// structure's LDS share, agents per CU or stage rounds change; no parity case holds more than 22.
#ifndef MPCX_MAXF
#define MPCX_MAXF 48
#endif
constexpr int MAXF = MPCX_MAXF;
static_assert(MAXF >= 1 && MAXF <= 64, "the filter test reads one entry per lane");
#ifndef MPCX_FSPILL
#define MPCX_FSPILL (1024 - MPCX_MAXF)
#endif
constexpr int FSPILL = MPCX_FSPILL;
static_assert(FSPILL >= 0, "spill list size");
constexpr double INF_BOUND = 1e19;
constexpr double TS = MPCX_TS;

// The phases of an IPM iteration are out-of-line calls in the fleet build (at 16 agents per CU
// a phase inlined into the loop keeps its operands live across the others: spills); the
// small-fleet build (one agent per CU, 512 VGPRs) inlines them into the kernel body, which
// removes the call overhead and the callee-saved register traffic from the single wave's chain
#ifndef MPCX_HOT  // (tests/test_native_abi.py compiles the phases out of line to inspect them)
#ifdef MPCX_WS_LDS
#define MPCX_HOT __attribute__((always_inline))
#else
#define MPCX_HOT __noinline__
#endif
#endif

// address-space qualified pointers: global_* / ds_* addressing inside the
// noinline phases (generic pointers compile to flat_*, which drain both
// counters and block load/store reordering)
typedef __attribute__((address_space(1))) double gdbl;
typedef __attribute__((address_space(1))) int gint;
typedef __attribute__((address_space(3))) double ldsd;
typedef __attribute__((address_space(3))) int ldsi;
// the agent's workspace slab: HBM (one slab per agent, 16 agents per CU) or, in the
// small-fleet variant (MPCX_WS_LDS: one agent per CU, fleets up to one agent per CU), LDS --
// every phase's operand round trip then costs an LDS access instead of an L2 / HBM one
#ifdef MPCX_WS_LDS
typedef ldsd wdbl;
typedef ldsi wint;
#else
typedef gdbl wdbl;
typedef gint wint;
#endif
typedef gdbl cdbl;  // the workspace's cold part (HBM in both builds)
typedef gint cint;

// stage-local system [V_k, lambda_rest | x_k | mu_k, x_{k+1} | rhs].  mu_k: the NMU
// continuity rows of the stage (the rows through x_{k+1}) when they are kept in the border
// (models with more states than free stage inputs): their multipliers join
// x_{k+1} in the chain block c_k = [mu_k, x_{k+1}] (indefinite 2x2-pivoted BK); otherwise
// NMU = 0 and every row is eliminated in the interior.
#ifndef MPCX_NMU
#define MPCX_NMU 0
#endif
constexpr int NMU = MPCX_NMU;
constexpr int NI = NV + NG - NMU;         // stage interior (eliminated in parallel)
constexpr int NXP = NX > 0 ? NX : 1;
constexpr int NXX = NXP * NXP;
constexpr int NC = NX + NMU;              // chain block per stage boundary
constexpr int NCP = NC > 0 ? NC : 1;
constexpr int NCC = NCP * NCP;
constexpr int SOFF = NXX + NCC + NCP * NXP;  // per stage: S00 (x_k), S11 (c_k), S10 (c_k x x_k)
constexpr int NLOC = NI + NX + NC;        // local system size
constexpr int RB = NLOC;                  // border row holding the right-hand side
constexpr int NTR = NX + NC + 1;          // trailing rows: x_k, c_k, border
constexpr int LMU = NI + NX;              // first local index of mu_k
constexpr int LX1 = NI + NX + NMU;        // first local index of x_{k+1}
static_assert(NMU <= NG, "bordered rows are stage rows");
constexpr int PKB = (NLOC + 1) * (NLOC + 2) / 2;  // packed lower triangle incl. border
constexpr int PKS = PKB | 1;              // odd stride between stage slots
static_assert(NI > 0, "stage interior must be non-empty");
#ifndef MPCX_CROW_INIT  // identity: rows in stage order after V
#define MPCX_CROW_INIT 0
#define MPCX_LROW_INIT 0
#endif
__constant__ int kCROW[NG > 0 ? NG : 1] = {MPCX_CROW_INIT};    // row r -> local index
__constant__ int kLROW[NLOC + 1] = {MPCX_LROW_INIT};           // local dual index -> row
static_assert(NLOC < 64, "local fixed-variable masks are 64-bit");
static_assert(N <= 64, "stage masks are 64-bit");
// Compact stage image (generated, runtime/codegen.py): only the structural nonzeros of the
// local system and the fill of the static elimination are stored.  Entry i < NLOC + 1 is
// the diagonal (i, i), entry CB + j the border (rhs) entry (RB, j), the rest follow in
// packed order; kCPK maps an entry to its packed dense index (dense fallback), kCIJ to
// (row | column << 8).  The evaluators write it (a.lp), the factorisation copies it to LDS.
constexpr int NCPT = MPCX_NCPT;
constexpr int NCS = NCPT | 1;             // odd stride between stage images
constexpr int CB = NLOC + 1;              // first border entry
static_assert(NCPT >= CB + NLOC, "compact image holds the diagonal and the border row");
__constant__ unsigned short kCPK[NCPT] = {MPCX_CPK_INIT};
__constant__ unsigned short kCIJ[NCPT] = {MPCX_CIJ_INIT};

// workspace layout (doubles per agent)
constexpr long O_X = 0, O_S = O_X + NW, O_LAM = O_S + M, O_ZL = O_LAM + M, O_ZU = O_ZL + NW;
constexpr long O_VL = O_ZU + NW, O_VU = O_VL + M, O_XL = O_VU + M, O_XU = O_XL + NW;
constexpr long O_SL = O_XU + NW, O_SU = O_SL + M, O_GS = O_SU + M, O_GV = O_GS + M;
constexpr long O_DX = O_GV + M, O_DS = O_DX + NW, O_DL = O_DS + M, O_LB = O_DL + M, O_UB = O_LB + M;
// hot part first (every iteration reads / writes it), then the cold part (scaling at init,
// the block-chain and dense fallbacks, the restoration phase): the small-fleet build keeps
// only the hot part in LDS
constexpr long O_SDG = O_UB + M;                 // [NL][N]      stage cost gradient
constexpr long O_JTL = O_SDG + (long)NL * N;     // [NL][N]      stage (gs*J)^T lambda
constexpr long O_RHS = O_JTL + (long)NL * N;     // [N][NB]      KKT right-hand side
constexpr long O_TR = O_RHS + (long)N * NB;      // [N][NTR][NI] back-substitution operators
constexpr long O_LP = O_TR + (long)N * NI * NTR;   // [NCPT][N] compact local systems (evaluators; stage-minor)
constexpr long O_DG = O_LP + (long)NCPT * N;       // [N][NLOC] diagonal terms (rhs phases; Newton mode)
constexpr long WS_HOT = O_DG + (long)N * NLOC;     // end of the hot part
constexpr long O_SDJ = WS_HOT;                   // [NG*NL][N]   stage jacobian (scaling, block chain)
constexpr long O_SDH = O_SDJ + (long)NG * NL * N;// [NL*NL][N]   stage hessian (block chain)
constexpr long O_PRM = O_SDH + (long)NL * NL * N;// [N][NI] ints interior pivot order (dense stages)
constexpr long O_KX = O_PRM + (long)N * NI;      // [N*NP] primal KKT diagonal   (block chain)
constexpr long O_KD = O_KX + (long)N * NP;       // [M] dual KKT diagonal        (block chain)
constexpr long O_SOL = O_KD + M;                 // [N][NB] solution             (block chain)
constexpr long O_FAC = O_SOL + (long)N * NB;     // [N][NB*LDB] block inverses   (block chain)
constexpr long O_CPL = O_FAC + (long)N * NB * LDB;  // [N][NB*NX] couplings      (block chain)
constexpr int SQ = NX > 0 ? NB : 1;   // the block-chain fallback exists only when stages are coupled
constexpr int SQL = NX > 0 ? LDB : 1;
constexpr long O_SQW = O_CPL + (long)N * NB * NXP;  // [2][SQ*SQL] block-chain inverse scratch W, Y
// feasibility restoration phase and soft restoration step (touched only on those paths)
constexpr long O_RP = O_SQW + (NX > 0 ? 2L * SQ * SQL : 0L);  // [M] restoration p (c~ - p + n)
constexpr long O_RN = O_RP + M;          // [M] restoration n
constexpr long O_RZP = O_RN + M;         // [M] bound multipliers of p
constexpr long O_RZN = O_RZP + M;        // [M] bound multipliers of n
constexpr long O_RDP = O_RZN + M;        // [M] Newton step of p
constexpr long O_RDN = O_RDP + M;        // [M] Newton step of n
constexpr long O_XR = O_RDN + M;         // [NW] x at the start of restoration (x_R) / soft-step backup
constexpr long O_SR = O_XR + NW;         // [M] slacks at the start of restoration / backup
constexpr long O_LR = O_SR + M;          // [M] multipliers backup (soft step)
constexpr long O_GVR = O_LR + M;         // [M] scaled constraint values backup (soft step)
constexpr long O_ZL0 = O_GVR + M;        // [NW] original bound multipliers at the start of restoration
constexpr long O_ZU0 = O_ZL0 + NW;
constexpr long O_VL0 = O_ZU0 + NW;       // [M]
constexpr long O_VU0 = O_VL0 + M;
constexpr long O_FLT0 = O_VU0 + M;       // [2][MAXF] the original filter while restoring
// iterative refinement of the restoration steps (resto_refine)
constexpr long O_RRHS = O_FLT0 + 2L * MAXF;      // [N][NB] the step's right-hand side
constexpr long O_RSOL = O_RRHS + (long)N * NB;   // [N][NB] the step so far
constexpr long O_RU = O_RSOL + (long)N * NB;     // [N][NLOC] local step vectors
constexpr long O_RY = O_RU + (long)N * NLOC;     // [N][NLOC] local KKT products
// filter spill lists: [tier][theta | phi][FSPILL], tier 0 the problem's filter (kept while a
// restoration phase runs), tier 1 the restoration phase's own
constexpr long O_FSP = O_RY + (long)N * NLOC;
constexpr long WS_DOUBLES = O_FSP + 4L * FSPILL;
// IPOPT restoration constants (its defaults; not exposed as options)
constexpr double RESTO_RHO = 1000.0;          // resto_penalty_parameter
constexpr double RESTO_KAPPA = 0.9;           // required_infeasibility_reduction
constexpr double SOFT_PD_FACTOR = 0.9999;     // soft_resto_pderror_reduction_factor
constexpr int MAX_SOFT_ITERS = 10;            // max_soft_resto_iters
constexpr double BOUND_MULT_RESET = 1000.0;   // bound_mult_reset_threshold
// PDFullSpaceSolver iterative refinement (IPOPT defaults)
constexpr int MIN_REFINE = 1;                 // min_refinement_steps
constexpr int MAX_REFINE = 10;                // max_refinement_steps
constexpr double RESID_RATIO_MAX = 1e-10;     // residual_ratio_max
constexpr double RESID_IMPROVE = 1.0;         // residual_improvement_factor
// factorisations one inertia correction may take: IPOPT bounds the shifts by delta_w_max only;
// two full shift sequences (x8 from delta_w_min to delta_w_max: 67 each, the second one with the
// constraint block regularised) fit
constexpr int IC_ATTEMPTS = 140;

using Args = mpcx_kernel_args;
// kernel arguments read in place from the kernarg segment (address space 4: scalar
// loads); passing the by-value kernel parameter by reference would make the
// compiler copy all of it (~400 B) into every lane's scratch
using KArgs = const __attribute__((address_space(4))) Args;
// wave-uniform 64-bit value into SGPRs
__device__ __forceinline__ unsigned long long uni64(unsigned long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// ---------------------------------------------------------------------------
// wave and lane-group helpers
// ---------------------------------------------------------------------------
// DPP lane exchange inside aligned groups (quad_perm xor1 / xor2, half-row and
// row mirrors): register-speed, no LDS round trip
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
// broadcast lane `l` (compile-time in unrolled loops) of a double: two v_readlane
__device__ __forceinline__ double rl_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
// Wave reductions (all 64 lanes active): DPP steps inside each row of 16 lanes (VALU
// latency), then the four row results read into SGPRs and combined -- instead of six
// LDS-permute (ds_bpermute) round trips.  MPCX_SHFL_REDUCE: the butterfly over __shfl_xor.
#ifndef MPCX_SHFL_REDUCE
__device__ __forceinline__ double wsum(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm xor 1
  v += dpp_f64<0x4E>(v);   // quad_perm xor 2
  v += dpp_f64<0x141>(v);  // row_half_mirror: the other quad of the half-row
  v += dpp_f64<0x140>(v);  // row_mirror: the other half of the row
  return (rl_f64(v, 0) + rl_f64(v, 16)) + (rl_f64(v, 32) + rl_f64(v, 48));
}
__device__ __forceinline__ double wmax(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  v = fmax(v, dpp_f64<0x140>(v));
  return fmax(fmax(rl_f64(v, 0), rl_f64(v, 16)), fmax(rl_f64(v, 32), rl_f64(v, 48)));
}
__device__ __forceinline__ double wmin(double v) {
  v = fmin(v, dpp_f64<0xB1>(v));
  v = fmin(v, dpp_f64<0x4E>(v));
  v = fmin(v, dpp_f64<0x141>(v));
  v = fmin(v, dpp_f64<0x140>(v));
  return fmin(fmin(rl_f64(v, 0), rl_f64(v, 16)), fmin(rl_f64(v, 32), rl_f64(v, 48)));
}
__device__ __forceinline__ int wsumi(int v) {
  v += dpp_i32<0xB1>(v);
  v += dpp_i32<0x4E>(v);
  v += dpp_i32<0x141>(v);
  v += dpp_i32<0x140>(v);
  return (__builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16)) +
         (__builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48));
}
#else
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, WAVE));
  return v;
}
__device__ __forceinline__ double wmin(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, WAVE));
  return v;
}
__device__ __forceinline__ int wsumi(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}
#endif
// argmax with smallest index on ties
__device__ __forceinline__ void wargmax(double& v, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ov = __shfl_xor(v, o, WAVE);
    int oi = __shfl_xor(idx, o, WAVE);
    if (ov > v || (ov == v && oi >= 0 && (idx < 0 || oi < idx))) { v = ov; idx = oi; }
  }
}
__device__ __forceinline__ void sync() { __syncthreads(); }
// Wavefront-scope sync for LDS-only hand-offs between lanes: a workgroup is one
// wavefront and the LDS executes one wave's DS instructions in issue order, so
// only compiler ordering is needed (no s_barrier, no vmcnt drain).
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lane id that the compiler can neither hoist nor keep live across calls: non-leaf phase
// functions recompute lane-derived values after each call instead of parking them in
// callee-saved VGPRs (saved to scratch on every call)
__device__ __forceinline__ int lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l & (WAVE - 1);  // the range for the compiler: lane-derived offsets are known non-negative
}

// Pin a loaded operand: the empty asm "uses" it here, so the compiler issues the load before this
// point instead of sinking it into the branch that uses it -- a load waited for inside a branch
// drains every older load (vmcnt counts in issue order), one memory round trip per such load.  A
// phase loads all its operands, pins them, then computes: one round trip for the batch.
#ifndef MPCX_NO_PIN
#define MPCX_PIN(x) asm volatile("" ::"v"(x))
#else  // diagnostics (A/B): the compiler places the loads
#define MPCX_PIN(x) (void)0
#endif
// The iteration head (inlined into the kernel body) is left to the compiler's placement: pinned as
// one batch it measured no faster at 4096 C3 agents and 0.5-1.5 % slower on C1 and MHE (r06/s6);
// MPCX_PIN_HEAD_BATCH pins it (A/B)
#ifdef MPCX_PIN_HEAD_BATCH
#define MPCX_PIN_HEAD(x) MPCX_PIN(x)
#else
#define MPCX_PIN_HEAD(x) (void)0
#endif

template <int GG>
__device__ __forceinline__ double gmax(double v) {
  if constexpr (GG >= 2) v = fmax(v, dpp_f64<0xB1>(v));
  if constexpr (GG >= 4) v = fmax(v, dpp_f64<0x4E>(v));
  if constexpr (GG >= 8) v = fmax(v, dpp_f64<0x141>(v));
  if constexpr (GG >= 16) v = fmax(v, dpp_f64<0x140>(v));
  if constexpr (GG >= 32) v = fmax(v, __shfl_xor(v, 16, WAVE));
  if constexpr (GG >= 64) v = fmax(v, __shfl_xor(v, 32, WAVE));
  return v;
}
__device__ __forceinline__ void amax_merge(double& v, int& idx, double ov, int oi) {
  if (ov > v || (ov == v && oi >= 0 && (idx < 0 || oi < idx))) { v = ov; idx = oi; }
}
template <int GG>
__device__ __forceinline__ void gargmax(double& v, int& idx) {
  if constexpr (GG >= 2) amax_merge(v, idx, dpp_f64<0xB1>(v), dpp_i32<0xB1>(idx));
  if constexpr (GG >= 4) amax_merge(v, idx, dpp_f64<0x4E>(v), dpp_i32<0x4E>(idx));
  if constexpr (GG >= 8) amax_merge(v, idx, dpp_f64<0x141>(v), dpp_i32<0x141>(idx));
  if constexpr (GG >= 16) amax_merge(v, idx, dpp_f64<0x140>(v), dpp_i32<0x140>(idx));
  if constexpr (GG >= 32) amax_merge(v, idx, __shfl_xor(v, 16, WAVE), __shfl_xor(idx, 16, WAVE));
  if constexpr (GG >= 64) amax_merge(v, idx, __shfl_xor(v, 32, WAVE), __shfl_xor(idx, 32, WAVE));
}

__device__ __forceinline__ bool isfin(double v) { return fabs(v) < INFINITY; }
__device__ __forceinline__ double absn(double v) {  // |v| with NaN -> +inf (total order for pivoting)
  const double t = fabs(v);
  return t == t ? t : INFINITY;
}

// ---------------------------------------------------------------------------
// LDS layout
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int pow2floor(int v) { int p = 1; while (p * 2 <= v) p *= 2; return p; }
__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }

// per-iteration results kept in LDS across the phase calls
struct OptErr {
  double dual, dual_u, primal, viol_u, pmx, pmn, s_d, s_c;
  int ncompl;
  __device__ double compl_at(double mu) const { return ncompl > 0 ? fmax(pmx - mu, mu - pmn) : 0.0; }
  __device__ double err_at(double mu) const { return fmax(fmax(dual / s_d, primal), compl_at(mu) / s_c); }
};

struct StepInfo {
  double amax, az, gphid, theta, barrier;
};

struct Trial {
  double f, theta, phi, fr;  // fr: restoration objective (restoration phase)
};

struct LSResult {
  Trial tr;
  double alpha;
  double bar;  // barrier sum (sum of log slacks) at the last trial point
  int accepted, ftype, trials;
};

struct Acceptable {
  double curr_f, last_f;
  int last_it, count;
};

// kernel loop state (uniform; every lane writes the same values)
struct KState {
  OptErr e0;       // optimality error at the current iterate
  Acceptable acc;  // acceptable-level counter
  StepInfo st;     // last recovered step
  LSResult ls;     // last line search
  double mu, tau, dw_last, fx, obj_scale, theta_max, theta_min, dw, dc, amin, barx;
  int nfilt, it, status, square, n_fact, n_ic, n_fallback, n_trials, n_chain, n_dense;
  // soft restoration / feasibility restoration phase (IPOPT BacktrackingLineSearch,
  // MinC_1NrmRestorationPhase): the original problem's state while restoring
  Acceptable acc0;
  double fo, zeta, prox, mu0, tau0, dw_last0, theta_max0, theta_min0, theta_start;
  int resto, soft, soft_count, lsmode, nfilt0, square_r, n_soft, n_resto_it;
  int n_filt_over, n_refine;  // filter insertions that dropped the oldest entry; refinement steps
  int nsp[2];                 // entries in the filter spill lists (tier 0: the problem's, 1: restoration's)
  double rnrm;                // refinement: max-norm of the step's full right-hand side
  // the barrier sum at the current iterate when it is the last accepted line-search trial point
  // (bar_ok): recover_step then takes it instead of recomputing every log of the slacks
  double bar_val;
  int bar_ok;
  double sw_l, sw_r;          // the line search's switching-condition powers (loop invariant)
};

#ifndef MPCX_NETX
#define MPCX_NETX 0
#define MPCX_NETO 0
#endif
// everything in LDS except the phase-shared union
struct LdsRest {
  double par[NPAR];        // agent parameters (read by every evaluation)
  double S[N * SOFF];      // local Schur blocks per stage: S00 (x_k), S11 (c_k), S10 (c_k x x_k)
  double Dinv[N * NCC];    // inverses of the chain pivots
  double zx[N * (NX + NCP)];  // forward-eliminated rhs of (x_k, c_k) per stage
  double xs[N * NCP];      // chain rhs, then solution (c_0 .. c_{N-1})
  double C[NCC];
  double CW[NCC];
  double CY[NCC];
  unsigned long long fixm[N];  // per stage: local primal indices that are fixed variables
  unsigned int ecls[WAVE];     // per lane: its rows' classes (2 bits per slot) and its variables' free /
                               // finite-bound bits (3 bits per slot, after them): cls_word, vcls_word
  int cperm[NCP];
  int cpiv[NCP];
  int fin[4];              // factor(): summed interior inertia (pos, neg, zero) and singular flag
  unsigned int dmask[2];   // factor(): stages the static plan rejected (dense path)
  int seq;                 // 1: last factorisation used the block chain
  int want_sdh;            // 1: keep the strided stage Hessians (block chain in use)
  int sdh_ok;              // 1: the workspace Hessians match the last eval_hess
  double hsig;             // sigma of the last eval_hess
  double fth[MAXF];
  double fph[MAXF];
#ifdef MPCX_NET_MFMA
  double netx[MPCX_NETX];  // network inputs of every call site (stage-major)
  double neto[MPCX_NETO];  // network values / derivatives of the current evaluation
#endif
  KState ks;
  // the kernarg segment and the agent's workspace slab, written once by the kernel: the
  // phases read them here (into SGPRs) instead of taking pointer arguments, which the calling
  // convention passes in VGPRs, callee-saved -- spilled to scratch -- when live across a call
  // (the kernarg segment pointer itself is not an implicit input of called functions)
  unsigned long long kp_bits, ws_bits;
#ifdef MPCX_TRACE_LS
  int trace_agent;         // the agent this workgroup solves (mapped launches: not blockIdx.x)
#endif
#ifdef MPCX_PROFILE
  double sprof[10];  // 0-3 factor, 4-5 solve, 6-9 iteration head (profile build)
  unsigned int dense_seen[2];  // stages ever rejected by the static plan (profile build)
#endif
};

// phase-shared union: block-chain fallback (its inverse scratch W, Y lives in the
// workspace), static compact images, dense images, Newton step, line-search trial point
struct SeqLds {
  double A[SQ * SQL];
  double B[SQ * NXP];
  double BP[SQ * NXP];
  double P[NXX];
  double v[SQ];
  double y[SQ];
  double t[SQ];
  int perm[SQ];
  int piv[SQ];
};
struct TrialLds {
  double xt[NW];
  double gt[MM];
};

// LDS budget (one wavefront per workgroup, 160 KB per CU): the most agents per CU for which
// the fixed part plus a minimal union fits -- all N compact stage images in one round if
// that still gives >= 4 agents per CU, else at least two images per round -- and the
// static rounds / dense images take what is left of that share.
constexpr int SLOT_BYTES = 8 * PKS + 8 * NI;  // dense packed system + perm/piv (fallback)
constexpr int CSLOT_BYTES = 8 * NCS;          // compact image (static elimination)
constexpr int REST_BYTES = (int)sizeof(LdsRest);
constexpr int UFIX_BYTES = cmax((int)sizeof(SeqLds), cmax(8 * N * NB, (int)sizeof(TrialLds)));
constexpr int LDS_CU_ALL = 163840, LDS_SLACK = 256;
#ifdef MPCX_WS_LDS
constexpr int WS_LDS_BYTES = (int)(8 * WS_HOT);
#else
constexpr int WS_LDS_BYTES = 0;
#endif
constexpr int LDS_CU = LDS_CU_ALL - WS_LDS_BYTES;  // what the per-agent LDS state may take
__host__ __device__ constexpr int apc_for(int need) {  // agents per CU for a per-agent need
  return (need + LDS_SLACK) * 16 <= LDS_CU ? 16 : (need + LDS_SLACK) * 8 <= LDS_CU ? 8
       : (need + LDS_SLACK) * 5 <= LDS_CU ? 5 : (need + LDS_SLACK) * 4 <= LDS_CU ? 4
       : (need + LDS_SLACK) * 3 <= LDS_CU ? 3 : (need + LDS_SLACK) * 2 <= LDS_CU ? 2 : 1;
}
#ifdef MPCX_STATIC_ELIM0
constexpr int K0 = 1;
#else
constexpr int K0 = 0;
#endif
constexpr int NRS = N - K0;                         // stages in the regular rounds
constexpr int APC_ONE = apc_for(REST_BYTES + cmax(UFIX_BYTES, cmax(SLOT_BYTES, cmax(NRS, 1) * CSLOT_BYTES)));
constexpr int APC_TWO = apc_for(REST_BYTES + cmax(UFIX_BYTES, cmax(SLOT_BYTES, cmin(cmax(NRS, 1), 2) * CSLOT_BYTES)));
#ifdef MPCX_WS_LDS
static_assert(WS_LDS_BYTES + REST_BYTES + UFIX_BYTES + LDS_SLACK <= LDS_CU_ALL, "MPCX_WS_LDS: workspace does not fit LDS");
constexpr int APC = 1;
#elif defined(MPCX_APC)  // agents per CU chosen by the build (more than 16: 5-8 waves per SIMD)
constexpr int APC = MPCX_APC;
#else
constexpr int APC = (APC_TWO >= 16 || APC_ONE < 4) ? APC_TWO : APC_ONE;
#endif
#ifdef MPCX_LDS_TARGET_OVERRIDE  // diagnostics (scripts/variants.py): per-agent byte budget
constexpr int LDS_BUDGET = MPCX_LDS_TARGET_OVERRIDE;
#else
constexpr int LDS_BUDGET = LDS_CU / APC - LDS_SLACK;
#endif
// static path: SRC compact images per round, one lane eliminates a stage, GC lanes assemble it.
// A model whose stage 0 opens rows that are equalities later on (MHE) has a second plan for
// stage 0 (gen_stage_elim0), run in a round of its own after stages K0.. so that no round
// executes both bodies divergently.
constexpr int SRC0 = cmax(1, cmin(cmin(cmax(NRS, 1), WAVE), (LDS_BUDGET - REST_BYTES) / CSLOT_BYTES));
constexpr int CROUNDS = (NRS + SRC0 - 1) / SRC0;
constexpr int SRC = CROUNDS > 0 ? (NRS + CROUNDS - 1) / CROUNDS : 1;  // stages per round (balanced)
constexpr int GC = pow2floor(WAVE / SRC);          // lanes per stage (assembly)
// dense Bunch-Kaufman path (stages the static plan rejects): SR dense images per round
constexpr int SR0 = cmax(1, cmin(cmin(N, WAVE), (LDS_BUDGET - REST_BYTES) / SLOT_BYTES));
constexpr int ROUNDS = (N + SR0 - 1) / SR0;
constexpr int SR = (N + ROUNDS - 1) / ROUNDS;   // stages per round (balanced)
constexpr int G = pow2floor(WAVE / SR);         // lanes per stage

struct ParLds {
  double F[SR * PKS];
  int perm[SR * NI];
  int piv[SR * NI];
};
struct ParCLds {
  double F[SRC * NCS];
};
union LinLds {
  SeqLds s;
  ParLds p;
  ParCLds c;
  double sol[N * NB];   // Newton step, block order [V, X1, lambda] per stage
  TrialLds t;           // line-search trial point (x, scaled g)
};

struct Lds : LdsRest {
  LinLds u;
};
#ifndef MPCX_LDS_TARGET_OVERRIDE
static_assert(sizeof(Lds) + LDS_SLACK <= LDS_CU / APC, "LDS share per agent exceeded");
#endif
// Waves per SIMD the LDS share allows (APC agents = APC one-wave workgroups per CU, 4 SIMDs):
// the register budget of the kernel and of every phase it calls follows it -- 128 VGPRs at
// 16 agents per CU, 512 at 4 (MHE: 480 -> 48 B/lane of call-frame scratch).  A tighter budget
// than the occupancy needs only spills (MPCX_MIN_WAVES overrides, scripts/variants.py).
#ifdef MPCX_MIN_WAVES
constexpr int MIN_WAVES = MPCX_MIN_WAVES;
#else
constexpr int MIN_WAVES = (APC + 3) / 4;
#endif

__shared__ Lds gL;  // one agent per workgroup: the agent's LDS scratch
__device__ __forceinline__ KArgs* kargs() { return (KArgs*)uni64(gL.kp_bits); }
#ifdef MPCX_WS_LDS
__shared__ double gWS[WS_HOT];
__device__ __forceinline__ wdbl* ws_base() { return (wdbl*)gWS; }
#else
__device__ __forceinline__ wdbl* ws_base() { return (wdbl*)uni64(gL.ws_bits); }
#endif
// the cold part: offsets >= WS_HOT of the agent's HBM slab (both builds)
__device__ __forceinline__ cdbl* cold_base() { return (cdbl*)uni64(gL.ws_bits); }
#define LDSP(x) ((ldsd*)(x))
#define LDSI(x) ((ldsi*)(x))
#ifdef MPCX_PROFILE
#define SPROF_DECL unsigned long long _st = __builtin_amdgcn_s_memtime();
#define SPROF(i) do { const unsigned long long _n = __builtin_amdgcn_s_memtime(); if (lane_now() == 0) gL.sprof[i] += (double)(_n - _st); _st = _n; } while (0)
#else
#define SPROF_DECL
#define SPROF(i) do { } while (0)
#endif
// Diagnostic build only (-DMPCX_TRACE_LS, scripts/resto_diag.py): the last line search of
// each agent is written to lam_w (header: theta, phi, gphi'd, alpha_min, theta_min, theta_max,
// mu, filter size, then the filter pairs) and lam_g (per trial: alpha, theta, phi, filter
// test, acceptance, f-type) instead of the multipliers.
#ifdef MPCX_TRACE_LS
#define TRACE_LS_HEAD(argp)                                                                      \
  do {                                                                                           \
    if (lane_now() == 0 && (*argp).lam_w != nullptr) {                                           \
      gdbl* h = (gdbl*)(*argp).lam_w + (long)gL.trace_agent * NW;                                \
      const double hv[8] = {K.st.theta, K.fx - K.mu * K.st.barrier, K.st.gphid, K.amin,          \
                            K.theta_min, K.theta_max, K.mu, (double)K.nfilt};                    \
      for (int q = 0; q < 8 && q < NW; ++q) h[q] = hv[q];                                        \
      for (int j = 0; j < K.nfilt && 10 + 2 * j + 1 < NW; ++j) { h[10 + 2 * j] = gL.fth[j]; h[11 + 2 * j] = gL.fph[j]; } \
      if (NW > 9) { h[8] = K.dw; h[9] = K.dc; }                                                  \
    }                                                                                            \
  } while (0)
#define TRACE_LS_TRIAL(argp, alpha, tr, okf, okt, ft)                                            \
  do {                                                                                           \
    const int t_ = K.ls.trials - 1;                                                              \
    if (lane_now() == 0 && (*argp).lam_g != nullptr && 6 * t_ + 5 < M) {                         \
      gdbl* g = (gdbl*)(*argp).lam_g + (long)gL.trace_agent * M + 6 * t_;                        \
      g[0] = (alpha); g[1] = (tr).theta; g[2] = (tr).phi; g[3] = (okf); g[4] = (okt); g[5] = (ft); \
    }                                                                                            \
  } while (0)
#else
#define TRACE_LS_HEAD(argp) do { } while (0)
#define TRACE_LS_TRIAL(argp, alpha, tr, okf, okt, ft) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// per-agent view: the workspace slab (wave-uniform, from LDS into SGPRs); lanes by lane_now()
// ---------------------------------------------------------------------------
struct Agent {
  // the agent's workspace slab, wave-uniform (SGPRs): nothing of the view is passed in VGPRs
  __device__ __forceinline__ wdbl* base() const { return ws_base(); }
  __device__ __forceinline__ cdbl* cold() const { return cold_base(); }
#define ws base()
  __device__ wdbl* x() const { return ws + O_X; }
  __device__ wdbl* s() const { return ws + O_S; }
  __device__ wdbl* lam() const { return ws + O_LAM; }
  __device__ wdbl* zL() const { return ws + O_ZL; }
  __device__ wdbl* zU() const { return ws + O_ZU; }
  __device__ wdbl* vL() const { return ws + O_VL; }
  __device__ wdbl* vU() const { return ws + O_VU; }
  __device__ wdbl* xL() const { return ws + O_XL; }
  __device__ wdbl* xU() const { return ws + O_XU; }
  __device__ wdbl* sL() const { return ws + O_SL; }
  __device__ wdbl* sU() const { return ws + O_SU; }
  __device__ wdbl* gs() const { return ws + O_GS; }
  __device__ wdbl* gv() const { return ws + O_GV; }
  __device__ wdbl* dx() const { return ws + O_DX; }
  __device__ wdbl* ds() const { return ws + O_DS; }
  __device__ wdbl* dl() const { return ws + O_DL; }
  __device__ wdbl* lb() const { return ws + O_LB; }
  __device__ wdbl* ub() const { return ws + O_UB; }
  __device__ wdbl* sdg() const { return ws + O_SDG; }
  __device__ wdbl* jtl() const { return ws + O_JTL; }
  __device__ cdbl* sdj() const { return cold_base() + O_SDJ; }
  __device__ cdbl* sdh() const { return cold_base() + O_SDH; }
  __device__ wdbl* rhs(int k) const { return ws + O_RHS + (long)k * NB; }
  __device__ wdbl* tr(int k) const { return ws + O_TR + k; }  // [NTR][NI][N]: W_k[t][p] at tr(k)[(t NI + p) N]
  __device__ cint* prm(int k) const { return reinterpret_cast<cint*>(cold_base() + O_PRM) + (long)k * NI; }
  __device__ cdbl* kx() const { return cold_base() + O_KX; }
  __device__ cdbl* kd() const { return cold_base() + O_KD; }
  __device__ cdbl* sol(int k) const { return cold_base() + O_SOL + (long)k * NB; }
  __device__ cdbl* fac(int k) const { return cold_base() + O_FAC + (long)k * NB * LDB; }
  __device__ cdbl* cpl(int k) const { return cold_base() + O_CPL + (long)k * NB * NXP; }
  __device__ wdbl* lp(int k) const { return ws + O_LP + k; }  // entry c of stage k at lp(k)[c * N]
  __device__ wdbl* dg(int k) const { return ws + O_DG + (long)k * NLOC; }
  __device__ cdbl* sqw() const { return cold_base() + O_SQW; }
  __device__ cdbl* rp() const { return cold_base() + O_RP; }
  __device__ cdbl* rn() const { return cold_base() + O_RN; }
  __device__ cdbl* rzp() const { return cold_base() + O_RZP; }
  __device__ cdbl* rzn() const { return cold_base() + O_RZN; }
  __device__ cdbl* rdp() const { return cold_base() + O_RDP; }
  __device__ cdbl* rdn() const { return cold_base() + O_RDN; }
  __device__ cdbl* xr() const { return cold_base() + O_XR; }
  __device__ cdbl* sr() const { return cold_base() + O_SR; }
  __device__ cdbl* lr() const { return cold_base() + O_LR; }
  __device__ cdbl* gvr() const { return cold_base() + O_GVR; }
  __device__ cdbl* zl0() const { return cold_base() + O_ZL0; }
  __device__ cdbl* zu0() const { return cold_base() + O_ZU0; }
  __device__ cdbl* vl0() const { return cold_base() + O_VL0; }
  __device__ cdbl* vu0() const { return cold_base() + O_VU0; }
  __device__ cdbl* flt0() const { return cold_base() + O_FLT0; }
  __device__ cdbl* fsp(int tier) const { return cold_base() + O_FSP + 2L * FSPILL * tier; }
  __device__ cdbl* rrhs() const { return cold_base() + O_RRHS; }
  __device__ cdbl* rsol() const { return cold_base() + O_RSOL; }
  __device__ cdbl* ru() const { return cold_base() + O_RU; }
  __device__ cdbl* ry() const { return cold_base() + O_RY; }
#undef ws
};

// constraint classes: 0 equality, 1 inequality with a finite bound, 2 free
__device__ __forceinline__ int cls_of(double lo, double hi, double sl, double su) {
  if (lo == hi) return 0;
  if (!isfin(sl) && !isfin(su)) return 2;
  return 1;
}
// The classes of a lane's rows (slot sl: row lane + 64 sl), computed once by init_agent (the bounds
// never change): the hot phases read one LDS word instead of loading ub to classify each row, and
// no row's class waits for its bound loads (r06: the iteration head classified a slot's rows from
// lb / ub before loading its other operands -- one more memory round trip per slot)
static_assert(2 * CS + 3 * VS <= 32, "element classes: 2 bits per constraint slot, 3 per variable slot, one word");
__device__ __forceinline__ unsigned cls_word() { return gL.ecls[lane_now()]; }
__device__ __forceinline__ int cls_slot(unsigned w, int sl) { return (int)((w >> (2 * sl)) & 3u); }
// The same for the variables (slot sl: variable lane + 64 sl): VFREE (NX <= i < NW, lo != hi),
// VLO / VHI (finite lower / upper bound), 3 bits per slot -- the hot phases' branches on a variable's
// bounds then do not wait for the bound loads (the compiler issued a slot's other loads only after
// testing lo == hi: two memory round trips per slot)
constexpr unsigned VFREE = 1u, VLO = 2u, VHI = 4u;
__device__ __forceinline__ unsigned vcls_word() { return gL.ecls[lane_now()] >> (2 * CS); }
__device__ __forceinline__ unsigned vcls_slot(unsigned w, int sl) { return (w >> (3 * sl)) & 7u; }

// ---------------------------------------------------------------------------
// evaluation (lane k evaluates stage k; parameters from LDS)
// ---------------------------------------------------------------------------
__device__ __forceinline__ const double* par_stage(int k) { return (const double*)(gL.par + NPG + k * NPS); }
__device__ __forceinline__ const double* par_global() { return (const double*)gL.par; }

// Network models (MPCX_NET_MFMA, runtime/codegen.py): before the stage functions run, the
// wave evaluates every network call site of every stage at the point on the matrix cores
// (csrc/mpcx_net_mfma.h): one lane per stage writes the inputs (gen_stage_netin), the
// wave runs gen_net_<kind>, and the stage functions read the entries they use from LDS.
#ifdef MPCX_NET_MFMA
#define NET_PREP(pt, kind)                                                                  \
  do {                                                                                      \
    for (int k = lane_now(); k < N; k += WAVE)                                                  \
      gen_stage_netin((const double*)((pt) + k * NP), par_stage(k), par_global(), k * TS,   \
                      (double*)gL.netx, k);                                                 \
    wsync();                                                                                \
    gen_net_##kind(LDSP(gL.netx), LDSP(gL.neto), lane_now());                               \
    wsync();                                                                                \
  } while (0)
#define STAGE_FG(...) gen_stage_fg_m(__VA_ARGS__, (const double*)gL.neto, k)
#define STAGE_GJ(...) gen_stage_gj_m(__VA_ARGS__, (const double*)gL.neto, k)
#define STAGE_HESS(...) gen_stage_hess_m(__VA_ARGS__, (const double*)gL.neto, k)
#else
#define NET_PREP(pt, kind) do { } while (0)
#define STAGE_FG(...) gen_stage_fg(__VA_ARGS__)
#define STAGE_GJ(...) gen_stage_gj(__VA_ARGS__)
#define STAGE_HESS(...) gen_stage_hess(__VA_ARGS__)
#endif

// f and unscaled g at the trial point in LDS (xt -> gt); returns wave-summed f
__device__ MPCX_HOT double eval_fg_lds(const Agent a) {
  NET_PREP(gL.u.t.xt, fg);
  double f = 0.0;
  for (int k = lane_now(); k < N; k += WAVE) {
    double fk = 0.0;
    STAGE_FG((const double*)(gL.u.t.xt + k * NP), par_stage(k), par_global(), k * TS, &fk,
             (double*)(gL.u.t.gt + k * NG), 1);
    f += fk;
  }
  return wsum(f);
}

// f and unscaled g at a point in the workspace
__device__ __noinline__ double eval_fg_ws(const Agent a, const wdbl* xv, wdbl* gout) {
  NET_PREP(xv, fg);
  double f = 0.0;
  for (int k = lane_now(); k < N; k += WAVE) {
    double fk = 0.0;
    STAGE_FG((const double*)(xv + k * NP), par_stage(k), par_global(), k * TS, &fk, (double*)(gout + k * NG), 1);
    f += fk;
  }
  return wsum(f);
}

// derivatives at a point in the workspace; full: also the strided jacobian (scaling and
// the block-chain fallback read it; the stage-parallel path reads lp and jtl only)
__device__ __noinline__ void eval_gj_ws(const Agent a, const wdbl* xv, int full) {
  NET_PREP(xv, gj);
  for (int k = lane_now(); k < N; k += WAVE)
    STAGE_GJ((const double*)(xv + k * NP), par_stage(k), par_global(), k * TS, (double*)(a.sdg() + k),
             (double*)(a.sdj() + k), N, (const double*)(a.gs() + k * NG), (double*)a.lp(k),
             (const double*)(a.lam() + k * NG), (double*)(a.jtl() + k), full);
}

// derivatives at the accepted trial point (still in LDS), with the accepted multipliers
// inlined into the kernel body: as a leaf call it saved and restored the callee-saved VGPRs
// its generated derivative code uses on every iteration (C3 -4 %, profiles/r03/s2/var_sgpr_c3.txt)
__device__ __attribute__((always_inline)) void eval_gj_lds(const Agent a) {
  NET_PREP(gL.u.t.xt, gj);
  const int full = gL.want_sdh;
  for (int k = lane_now(); k < N; k += WAVE)
    STAGE_GJ((const double*)(gL.u.t.xt + k * NP), par_stage(k), par_global(), k * TS,
             (double*)(a.sdg() + k), (double*)(a.sdj() + k), N, (const double*)(a.gs() + k * NG),
             (double*)a.lp(k), (const double*)(a.lam() + k * NG), (double*)(a.jtl() + k), full);
}

// Hessian of sigma*f + sum lam_i * gs_i * g_i (scaled Lagrangian) into the packed
// stage systems; the strided full Hessians (read only by the block-chain fallback)
// are written when that path is in use, or on demand (eval_hess_full)
__device__ MPCX_HOT void eval_hess_impl(const Agent a, double sigma, int full) {
  NET_PREP(a.x(), hess);
  for (int k = lane_now(); k < N; k += WAVE) {
    double lk[NG > 0 ? NG : 1];
#pragma unroll
    for (int r = 0; r < NG; ++r) lk[r] = a.lam()[k * NG + r] * a.gs()[k * NG + r];
    STAGE_HESS((const double*)(a.x() + k * NP), par_stage(k), par_global(), k * TS, sigma, lk,
               (double*)(a.sdh() + k), N, (double*)a.lp(k), full);
  }
  if (lane_now() == 0) { gL.hsig = sigma; gL.sdh_ok = full; }
}
__device__ __forceinline__ void eval_hess(const Agent a, double sigma) { eval_hess_impl(a, sigma, gL.want_sdh); }

// gradient of the (unscaled) objective w.r.t. w[i], i >= NX (stage derivatives of
// stage b and, for a state, the X0 part of stage b+1)
// Both loads are unconditional (the second from a valid address either way, its value selected
// away where unused): a load under a divergent branch is waited for inside the branch, and the
// wait drains every older load of the phase (vmcnt counts in issue order) -- r06: four such drains
// per iteration head, one memory round trip each
__device__ __forceinline__ double stage_pair_sum(const wdbl* arr, int i) {
  const int b = (i - NX) / NP, off = (i - NX) % NP;
  const int i0 = (NX + off) * N + b;
  const double v = arr[i0];
  if constexpr (NX > 0) {
    const bool two = off >= NV && b + 1 < N;
    const double w = arr[two ? (off - NV) * N + b + 1 : i0];
    return two ? v + w : v;
  }
  return v;
}
__device__ __forceinline__ double acc_grad(const Agent a, int i) { return stage_pair_sum(a.sdg(), i); }
// (J~^T lam)[i] with J~ = gs*J, from the per-stage products the evaluators wrote
__device__ __forceinline__ double acc_jtl(const Agent a, int i) { return stage_pair_sum(a.jtl(), i); }

// ---------------------------------------------------------------------------
// dense Bunch-Kaufman LDL^T in LDS (full symmetric storage, wave-wide):
// block-chain fallback and the nx x nx state-chain pivots
// ---------------------------------------------------------------------------
struct Inertia {
  int pos, neg, zero;
};

// zero pivots: absolute threshold (same constant as oracle/ipm.py ZERO_PIVOT);
// the barrier terms make the block norm unbounded near active bounds, so a
// norm-relative test would misclassify legitimate -delta_c pivots
constexpr double ZERO_PIVOT = 1e-20;
constexpr double BK_ALPHA = 0.6403882032022076;  // (1 + sqrt(17)) / 8

template <int NN, int LD>
__device__ __noinline__ Inertia bk_factor(ldsd* A, ldsi* perm, ldsi* piv, int lane) {
  constexpr int NN2 = NN * NN;
  Inertia in{0, 0, 0};
  for (int i = lane; i < NN; i += WAVE) perm[i] = i;
  wsync();
  int k = 0;
#pragma unroll 1
  while (k < NN) {
    const double akk = fabs(A[k * LD + k]);
    double lam = -1.0;
    int r = -1;
    for (int i = k + 1 + lane; i < NN; i += WAVE) {
      const double t = fabs(A[i * LD + k]);
      if (t > lam) { lam = t; r = i; }
    }
    if constexpr (NN <= 9) {  // candidates in lanes 0..7: DPP reduction inside the lane octet
      gargmax<8>(lam, r);
      lam = rl_f64(lam, 0);
      r = __builtin_amdgcn_readfirstlane(r);
    } else {
      wargmax(lam, r);
    }
    if (r < 0) lam = 0.0;
    int size = 1, kp = k;
    if (fmax(akk, lam) == 0.0 || akk >= BK_ALPHA * lam) {
      size = 1; kp = k;
    } else {
      double sg = 0.0;
      for (int j = k + lane; j < NN; j += WAVE)
        if (j != r) sg = fmax(sg, fabs(A[r * LD + j]));
      double sigma;
      if constexpr (NN <= 8) sigma = rl_f64(gmax<8>(sg), 0);
      else sigma = wmax(sg);
      if (akk * sigma >= BK_ALPHA * lam * lam) {
        size = 1; kp = k;
      } else if (fabs(A[r * LD + r]) >= BK_ALPHA * sigma) {
        size = 1; kp = r;
      } else {
        size = 2; kp = r;
      }
    }
    const int kk = k + size - 1;
    if (kp != kk) {
      for (int j = lane; j < NN; j += WAVE) {
        const double t = A[kp * LD + j]; A[kp * LD + j] = A[kk * LD + j]; A[kk * LD + j] = t;
      }
      wsync();
      for (int i = lane; i < NN; i += WAVE) {
        const double t = A[i * LD + kp]; A[i * LD + kp] = A[i * LD + kk]; A[i * LD + kk] = t;
      }
      if (lane == 0) { const int t = perm[kp]; perm[kp] = perm[kk]; perm[kk] = t; }
      wsync();
    }
    if (size == 1) {
      const double d = A[k * LD + k];
      if (fabs(d) <= ZERO_PIVOT) {
        in.zero++;
        for (int i = k + 1 + lane; i < NN; i += WAVE) A[i * LD + k] = 0.0;
      } else {
        if (d > 0) in.pos++; else in.neg++;
        const double rd = MPCX_RCP(d);
        for (int t = lane; t < NN2; t += WAVE) {
          const int i = t / NN, j = t % NN;
          if (i > k && j > k) A[i * LD + j] -= A[i * LD + k] * A[j * LD + k] * rd;
        }
        wsync();
        for (int i = k + 1 + lane; i < NN; i += WAVE) A[i * LD + k] *= rd;
      }
      if (lane == 0) piv[k] = 1;
    } else {
      const double a11 = A[k * LD + k], a21 = A[(k + 1) * LD + k], a22 = A[(k + 1) * LD + k + 1];
      const double det = a11 * a22 - a21 * a21;
      if (fabs(det) <= ZERO_PIVOT * ZERO_PIVOT) {
        in.zero += 2;
      } else {
        if (det < 0) { in.pos++; in.neg++; }
        else if (a11 + a22 > 0) in.pos += 2;
        else in.neg += 2;
      }
      const double rdet = MPCX_RCP(det);
      for (int t = lane; t < NN2; t += WAVE) {
        const int i = t / NN, j = t % NN;
        if (i > k + 1 && j > k + 1) {
          const double ai1 = A[i * LD + k], ai2 = A[i * LD + k + 1];
          const double l1 = (ai1 * a22 - ai2 * a21) * rdet, l2 = (ai2 * a11 - ai1 * a21) * rdet;
          A[i * LD + j] -= l1 * A[j * LD + k] + l2 * A[j * LD + k + 1];
        }
      }
      wsync();
      for (int i = k + 2 + lane; i < NN; i += WAVE) {
        const double ai1 = A[i * LD + k], ai2 = A[i * LD + k + 1];
        A[i * LD + k] = (ai1 * a22 - ai2 * a21) * rdet;
        A[i * LD + k + 1] = (ai2 * a11 - ai1 * a21) * rdet;
      }
      if (lane == 0) { piv[k] = 2; piv[k + 1] = 0; }
    }
    wsync();
    k += size;
  }
  return in;
}

// Explicit inverse of a factored block, A^{-1} = P^T L^{-T} D^{-1} L^{-1} P,
// written in the ORIGINAL index order to `out` (ld LD).  W, Y: scratch (LDS for the chain
// pivots, the workspace for the block-chain fallback).
template <int NN, int LD, typename OutT, typename WT>
__device__ __noinline__ void bk_inverse(const ldsd* A, const ldsi* perm, const ldsi* piv, WT* W,
                                        WT* Y, OutT* out, int lane) {
  constexpr int NN2 = NN * NN;
  for (int t = lane; t < NN2; t += WAVE) {
    const int i = t / NN, j = t % NN;
    W[i * LD + j] = (i == j) ? 1.0 : 0.0;
  }
  wsync();
  int k = 0;
#pragma unroll 1
  while (k < NN) {
    const int sz = piv[k];
    for (int t = lane; t < NN2; t += WAVE) {
      const int i = t / NN, j = t % NN;
      if (i >= k + sz && j <= k + sz - 1) {
        double v = A[i * LD + k] * W[k * LD + j];
        if (sz == 2) v += A[i * LD + k + 1] * W[(k + 1) * LD + j];
        W[i * LD + j] -= v;
      }
    }
    wsync();
    k += sz;
  }
  for (int t = lane; t < NN2; t += WAVE) {
    const int i = t / NN, j = t % NN;
    const int sz = piv[i];
    if (sz == 1) {
      const double d = A[i * LD + i];
      Y[i * LD + j] = (d != 0.0) ? W[i * LD + j] / d : 0.0;
    } else if (sz == 2) {
      const double a11 = A[i * LD + i], a21 = A[(i + 1) * LD + i], a22 = A[(i + 1) * LD + i + 1];
      const double det = a11 * a22 - a21 * a21;
      const double w0 = W[i * LD + j], w1 = W[(i + 1) * LD + j];
      Y[i * LD + j] = (a22 * w0 - a21 * w1) / det;
      Y[(i + 1) * LD + j] = (a11 * w1 - a21 * w0) / det;
    }
  }
  wsync();
  for (int t = lane; t < NN2; t += WAVE) {
    const int i = t / NN, j = t % NN;
    double acc = 0.0;
    const int mx = i > j ? i : j;
    for (int m = (mx > 0 ? mx - 1 : 0); m < NN; ++m) acc += W[m * LD + i] * Y[m * LD + j];
    out[perm[i] * LD + perm[j]] = acc;
  }
  wsync();
}

// Inverse AND inertia of a small symmetric indefinite block in one pass (state-chain
// pivots, NN*NN <= 64): the symmetric sweep operator (Goodnight) with Bunch-Kaufman pivot
// choices.  Lane (i, j) owns entry (i, j) of the LDS image; each pivot step is one pivot
// search (DPP reductions in the first lane octet) plus ONE read-modify-write of the whole
// block -- the swept rows/columns become the inverse as the sweep goes, so there are no
// row swaps, no separate L^{-1} sweep and no final product (bk_factor + bk_inverse take
// ~3x the dependent LDS round trips).  Pivots are the Schur-complement pivots of a
// symmetric elimination in the chosen order, so the inertia is the same (Sylvester); a
// zero pivot is counted and its row/column left out of the inverse, as the LDL^T path
// does.  A is destroyed; out receives A^{-1} (ld LD).
template <int NN, int LD, typename OutT>
__device__ __noinline__ Inertia bk_sweep(ldsd* A, OutT* out, int lane) {
  static_assert(NN * NN <= WAVE && NN <= 8, "one lane per entry; pivot candidates in one lane octet");
  constexpr unsigned FULL = (1u << NN) - 1u;
  Inertia in{0, 0, 0};
  const int ti = lane / NN, tj = lane % NN;
  const bool own = lane < NN * NN;
  unsigned done = 0u, zero = 0u;
#pragma unroll 1
  while (done != FULL) {
    const int k = __builtin_ctz(~done);
    const bool cand = lane < NN && !((done >> lane) & 1u);
    double lam = -1.0;
    int r = -1;
    if (cand && lane != k) { lam = fabs(A[lane * LD + k]); r = lane; }
    gargmax<8>(lam, r);
    lam = rl_f64(lam, 0);
    r = __builtin_amdgcn_readfirstlane(r);
    if (r < 0) lam = 0.0;
    const double akk = fabs(A[k * LD + k]);
    int p = k, q = -1;  // 1x1 pivot p, or 2x2 pivot {k, q}
    if (!(fmax(akk, lam) == 0.0 || akk >= BK_ALPHA * lam)) {
      double sg = 0.0;
      if (cand && lane != r) sg = fabs(A[r * LD + lane]);
      const double sigma = rl_f64(gmax<8>(sg), 0);
      if (akk * sigma >= BK_ALPHA * lam * lam) p = k;
      else if (fabs(A[r * LD + r]) >= BK_ALPHA * sigma) p = r;
      else q = r;
    }
    if (q < 0) {
      const double d = A[p * LD + p];
      done |= 1u << p;
      if (fabs(d) <= ZERO_PIVOT) { in.zero++; zero |= 1u << p; continue; }
      if (d > 0) in.pos++; else in.neg++;
      const double rd = MPCX_RCP(d);
      if (own) {
        const double aip = A[ti * LD + p], apj = A[p * LD + tj], aij = A[ti * LD + tj];
        A[ti * LD + tj] = (ti == p) ? ((tj == p) ? -rd : apj * rd) : (tj == p) ? aip * rd : aij - aip * apj * rd;
      }
    } else {
      const double a11 = A[k * LD + k], a21 = A[q * LD + k], a22 = A[q * LD + q];
      const double det = a11 * a22 - a21 * a21;
      done |= (1u << k) | (1u << q);
      if (fabs(det) <= ZERO_PIVOT * ZERO_PIVOT) { in.zero += 2; zero |= (1u << k) | (1u << q); continue; }
      if (det < 0) { in.pos++; in.neg++; }
      else if (a11 + a22 > 0) in.pos += 2;
      else in.neg += 2;
      const double rdet = MPCX_RCP(det);
      const double p11 = a22 * rdet, p12 = -a21 * rdet, p22 = a11 * rdet;  // pivot-block inverse
      if (own) {
        const double aik = A[ti * LD + k], aiq = A[ti * LD + q], akj = A[k * LD + tj], aqj = A[q * LD + tj];
        const double aij = A[ti * LD + tj];
        const double xk = aik * p11 + aiq * p12, xq = aik * p12 + aiq * p22;  // row i times P^{-1}
        const double yk = p11 * akj + p12 * aqj, yq = p12 * akj + p22 * aqj;  // P^{-1} times column j
        const bool ip = ti == k || ti == q, jp = tj == k || tj == q;
        double v;
        if (ip && jp) v = -((ti == k) ? ((tj == k) ? p11 : p12) : ((tj == k) ? p12 : p22));
        else if (ip) v = (ti == k) ? yk : yq;
        else if (jp) v = (tj == k) ? xk : xq;
        else v = aij - (xk * akj + xq * aqj);
        A[ti * LD + tj] = v;
      }
    }
    wsync();
  }
  wsync();
  if (own) out[ti * LD + tj] = (((zero >> ti) | (zero >> tj)) & 1u) ? 0.0 : -A[ti * LD + tj];
  wsync();
  return in;
}

// Two independent blocks swept at once (the twisted chain's forward and backward pivots, r04):
// bk_sweep's arithmetic and pivot choices for each block -- lanes 0-7 search block A's pivot
// candidates and lanes 8-15 block B's, each octet with its own DPP reduction, and every owning
// lane updates its entry of both blocks -- so one pass costs the dependent latency of one.
// In place (each block receives its own inverse); twob false sweeps A alone.
template <int NN, int LD>
__device__ __noinline__ Inertia bk_sweep2(ldsd* A, ldsd* B, bool twob, int lane) {
  static_assert(NN * NN <= WAVE && NN <= 8, "one lane per entry; pivot candidates in one lane octet");
  constexpr unsigned FULL = (1u << NN) - 1u;
  Inertia in{0, 0, 0};
  const int ti = lane / NN, tj = lane % NN;
  const bool own = lane < NN * NN;
  const int oc = lane >> 3, ol = lane & 7;  // octet 0 searches A, octet 1 searches B
  ldsd* const M = oc == 0 ? A : B;
  unsigned dA = 0u, zA = 0u, dB = twob ? 0u : FULL, zB = 0u;
#pragma unroll 1
  while (dA != FULL || dB != FULL) {
    const bool goA = dA != FULL, goB = dB != FULL;
    const int kA = goA ? __builtin_ctz(~dA) : 0, kB = goB ? __builtin_ctz(~dB) : 0;
    const int k = oc == 0 ? kA : kB;
    const bool cand = oc < 2 && ol < NN && (oc == 0 ? goA : goB) && !(((oc == 0 ? dA : dB) >> ol) & 1u);
    double lam = -1.0;
    int r = -1;
    if (cand && ol != k) { lam = fabs(M[ol * LD + k]); r = ol; }
    gargmax<8>(lam, r);
    double lamA = rl_f64(lam, 0), lamB = rl_f64(lam, 8);
    const int rA = __builtin_amdgcn_readlane(r, 0), rB = __builtin_amdgcn_readlane(r, 8);
    if (rA < 0) lamA = 0.0;
    if (rB < 0) lamB = 0.0;
    const double akkA = fabs(A[kA * LD + kA]), akkB = fabs(B[kB * LD + kB]);
    const bool needA = goA && !(fmax(akkA, lamA) == 0.0 || akkA >= BK_ALPHA * lamA);
    const bool needB = goB && !(fmax(akkB, lamB) == 0.0 || akkB >= BK_ALPHA * lamB);
    int pA = kA, qA = -1, pB = kB, qB = -1;
    if (needA || needB) {
      const int ro = oc == 0 ? rA : rB;
      double sg = 0.0;
      if (cand && ol != ro && (oc == 0 ? needA : needB)) sg = fabs(M[ro * LD + ol]);
      const double g8 = gmax<8>(sg);
      const double sigA = rl_f64(g8, 0), sigB = rl_f64(g8, 8);
      if (needA) {
        if (akkA * sigA >= BK_ALPHA * lamA * lamA) pA = kA;
        else if (fabs(A[rA * LD + rA]) >= BK_ALPHA * sigA) pA = rA;
        else qA = rA;
      }
      if (needB) {
        if (akkB * sigB >= BK_ALPHA * lamB * lamB) pB = kB;
        else if (fabs(B[rB * LD + rB]) >= BK_ALPHA * sigB) pB = rB;
        else qB = rB;
      }
    }
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
      if (blk == 0 ? !goA : !goB) continue;
      ldsd* const X = blk == 0 ? A : B;
      unsigned& done = blk == 0 ? dA : dB;
      unsigned& zero = blk == 0 ? zA : zB;
      const int kk = blk == 0 ? kA : kB, p = blk == 0 ? pA : pB, q = blk == 0 ? qA : qB;
      if (q < 0) {
        const double d = X[p * LD + p];
        done |= 1u << p;
        if (fabs(d) <= ZERO_PIVOT) { in.zero++; zero |= 1u << p; continue; }
        if (d > 0) in.pos++; else in.neg++;
        const double rd = MPCX_RCP(d);
        if (own) {
          const double aip = X[ti * LD + p], apj = X[p * LD + tj], aij = X[ti * LD + tj];
          X[ti * LD + tj] = (ti == p) ? ((tj == p) ? -rd : apj * rd) : (tj == p) ? aip * rd : aij - aip * apj * rd;
        }
      } else {
        const double a11 = X[kk * LD + kk], a21 = X[q * LD + kk], a22 = X[q * LD + q];
        const double det = a11 * a22 - a21 * a21;
        done |= (1u << kk) | (1u << q);
        if (fabs(det) <= ZERO_PIVOT * ZERO_PIVOT) { in.zero += 2; zero |= (1u << kk) | (1u << q); continue; }
        if (det < 0) { in.pos++; in.neg++; }
        else if (a11 + a22 > 0) in.pos += 2;
        else in.neg += 2;
        const double rdet = MPCX_RCP(det);
        const double p11 = a22 * rdet, p12 = -a21 * rdet, p22 = a11 * rdet;
        if (own) {
          const double aik = X[ti * LD + kk], aiq = X[ti * LD + q], akj = X[kk * LD + tj], aqj = X[q * LD + tj];
          const double aij = X[ti * LD + tj];
          const double xk = aik * p11 + aiq * p12, xq = aik * p12 + aiq * p22;
          const double yk = p11 * akj + p12 * aqj, yq = p12 * akj + p22 * aqj;
          const bool ip = ti == kk || ti == q, jp = tj == kk || tj == q;
          double v;
          if (ip && jp) v = -((ti == kk) ? ((tj == kk) ? p11 : p12) : ((tj == kk) ? p12 : p22));
          else if (ip) v = (ti == kk) ? yk : yq;
          else if (jp) v = (tj == kk) ? xk : xq;
          else v = aij - (xk * akj + xq * aqj);
          X[ti * LD + tj] = v;
        }
      }
    }
    wsync();
  }
  if (own) {
    A[ti * LD + tj] = (((zA >> ti) | (zA >> tj)) & 1u) ? 0.0 : -A[ti * LD + tj];
    if (twob) B[ti * LD + tj] = (((zB >> ti) | (zB >> tj)) & 1u) ? 0.0 : -B[ti * LD + tj];
  }
  wsync();
  return in;
}

// ---------------------------------------------------------------------------
// KKT entries
// ---------------------------------------------------------------------------
enum Mode { NEWTON = 0, LSQ = 1 };

struct KKTDiag {
  double dw, dc;
  Mode mode;
};

__device__ __forceinline__ double sigma_x_v(double xv, double lo, double hi, double zl, double zu) {
  if (lo == hi) return 0.0;
  double s = 0.0;
  if (isfin(lo)) s += zl / (xv - lo);
  if (isfin(hi)) s += zu / (hi - xv);
  return s;
}
__device__ __forceinline__ double sigma_s_v(double sv, double sl, double su, double vl, double vu) {
  double s = 0.0;
  if (isfin(sl)) s += vl / (sv - sl);
  if (isfin(su)) s += vu / (su - sv);
  return s;
}
__device__ __forceinline__ double dual_diag_v(int cl, double sig, const KKTDiag kd) {
  if (kd.mode == LSQ) return cl == 0 ? 0.0 : 1.0;
  if (cl == 0) return kd.dc;
  if (cl == 2) return 1.0;
  return 1.0 / (sig + kd.dw) + kd.dc;
}
// The per-iteration vector phases (iteration head, inertia-correction rhs, step recovery,
// accept) take ONE reciprocal per slack, 1 / (x - lo) and 1 / (hi - x), and multiply, where the
// formulas divide several numerators by the same slack (mu / s, z / s, Sigma = z / s, ...); the
// reciprocal is MPCX_RCP (v_rcp_f64 + two Newton steps, generated preamble).  The quotients agree
// with the divisions to an ulp or two; the oracle's decisions (statuses, iteration counts) are
// unchanged on every parity case (tests/test_gpu_ipm.py).  r05: a division is eleven dependent
// VALU instructions, and these phases held ~120 of them per iteration.
__device__ __forceinline__ double rcp_or0(bool fin, double s) { return fin ? MPCX_RCP(s) : 0.0; }

// ---------------------------------------------------------------------------
// sequential block chain (fallback when a stage interior is singular)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int crow(int r);
// per-variable / per-constraint diagonal terms (workspace; NaN in kx marks a fixed variable).
// Newton mode: the terms the rhs phases wrote (dg: barrier Sigma, the restoration's proximity
// weight and its eliminated p, n terms), + delta_w on the primal side
__device__ __noinline__ void kkt_diagonals(const Agent a, const KKTDiag kd) {
  for (int q = lane_now(); q < N * NP; q += WAVE) {
    const int i = NX + q, b = q / NP, off = q % NP;
    const double lo = a.xL()[i], hi = a.xU()[i];
    a.kx()[q] = (lo == hi) ? NAN : (kd.mode == LSQ ? 1.0 : a.dg(b)[off < NV ? off : LX1 + off - NV] + kd.dw);
  }
  for (int c = lane_now(); c < M; c += WAVE) {
    const double sl = a.sL()[c], su = a.sU()[c];
    const int cl = cls_of(a.lb()[c], a.ub()[c], sl, su);
    a.kd()[c] = kd.mode == LSQ ? dual_diag_v(cl, 0.0, kd) : -a.dg(c / NG)[crow(c % NG)];
  }
  sync();
}

__device__ __forceinline__ bool kfixed(const Agent a, int k, int q) {
  const double v = a.kx()[k * NP + q];
  return v != v;
}

// entry (i, j) of KKT block k = [V_k, X_{k+1}, lambda_k] (before the Schur update)
__device__ __forceinline__ double kkt_entry(const Agent a, int k, int i, int j, Mode mode) {
  if (i < NP && j < NP) {
    if (kfixed(a, k, i) || kfixed(a, k, j)) return (i == j) ? 1.0 : 0.0;
    if (mode == LSQ) return (i == j) ? 1.0 : 0.0;
    double v = a.sdh()[((NX + i) * NL + NX + j) * N + k];
    if (NX > 0 && i >= NV && j >= NV && k + 1 < N) v += a.sdh()[((i - NV) * NL + (j - NV)) * N + k + 1];
    if (i == j) v += a.kx()[k * NP + i];
    return v;
  }
  if (i >= NP && j >= NP) return (i == j) ? -a.kd()[k * NG + i - NP] : 0.0;
  const int r = (i >= NP) ? i - NP : j - NP;
  const int q = (i >= NP) ? j : i;
  if (kfixed(a, k, q)) return 0.0;
  return a.gs()[k * NG + r] * a.sdj()[(r * NL + NX + q) * N + k];
}

// coupling of block k (row) to x_k = X0 of stage k (column c < NX)
__device__ __forceinline__ double coupling(const Agent a, int k, int row, int c, Mode mode) {
  if (k == 0 || kfixed(a, k - 1, NV + c)) return 0.0;
  if (row < NP) {
    if (mode == LSQ || kfixed(a, k, row)) return 0.0;
    return a.sdh()[((NX + row) * NL + c) * N + k];
  }
  const int r = row - NP;
  return a.gs()[k * NG + r] * a.sdj()[(r * NL + c) * N + k];
}

constexpr int NB2 = NB * NB;
constexpr int EPL = (NB2 + WAVE - 1) / WAVE;  // block elements per lane

__device__ __noinline__ void seq_assemble(const Agent a, Mode mode) {
  for (int t = lane_now(); t < N * NB2; t += WAVE) {
    const int k = t / NB2, e = t % NB2, i = e / NB, j = e % NB;
    a.fac(k)[i * LDB + j] = kkt_entry(a, k, i, j, mode);
  }
  if (NX > 0) {
    for (int t = lane_now(); t < N * NB * NX; t += WAVE) {
      const int k = t / (NB * NX), e = t % (NB * NX);
      a.cpl(k)[e] = coupling(a, k, e / NX, e % NX, mode);
    }
  }
  sync();
}

// Block LDL^T through the state columns: D_k = A_k - B_k [D_{k-1}^{-1}]_{xx} B_k^T;
// each block's explicit inverse is stored (solves become mat-vecs).
__device__ __noinline__ Inertia seq_factor(const Agent a, const KKTDiag kd) {
  if constexpr (NX == 0) {
    return Inertia{0, 0, 1};
  } else {
    SeqLds& L = gL.u.s;
    const int lane = lane_now();
    Inertia in{0, 0, 0};
    kkt_diagonals(a, kd);
    seq_assemble(a, kd.mode);
    double pre[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int t = lane + e * WAVE;
      pre[e] = (t < NB2) ? a.fac(0)[(t / NB) * LDB + t % NB] : 0.0;
    }
#pragma unroll 1
    for (int k = 0; k < N; ++k) {
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int t = lane + e * WAVE;
        if (t < NB2) L.A[(t / NB) * LDB + t % NB] = pre[e];
      }
      if (k > 0)
        for (int t = lane; t < NB * NX; t += WAVE) L.B[t] = a.cpl(k)[t];
      sync();
      if (k + 1 < N) {  // prefetch block k+1 (consumed at the top of the next step)
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const int t = lane + e * WAVE;
          pre[e] = (t < NB2) ? a.fac(k + 1)[(t / NB) * LDB + t % NB] : 0.0;
        }
      }
      if (k > 0) {
        for (int t = lane; t < NB * NX; t += WAVE) {
          const int i = t / NX, d = t % NX;
          double s = 0.0;
          for (int c = 0; c < NX; ++c) s += L.B[i * NX + c] * L.P[c * NX + d];
          L.BP[t] = s;
        }
        wsync();
        for (int t = lane; t < NB2; t += WAVE) {
          const int i = t / NB, j = t % NB;
          double s = 0.0;
          for (int d = 0; d < NX; ++d) s += L.BP[i * NX + d] * L.B[j * NX + d];
          L.A[i * LDB + j] -= s;
        }
        wsync();
      }
      const Inertia bi = bk_factor<NB, LDB>(LDSP(L.A), LDSI(L.perm), LDSI(L.piv), lane);
      in.pos += bi.pos; in.neg += bi.neg; in.zero += bi.zero;
      bk_inverse<NB, LDB>(LDSP(L.A), LDSI(L.perm), LDSI(L.piv), a.sqw(), a.sqw() + SQ * SQL, a.fac(k), lane);
      sync();
      if (k + 1 < N)
        for (int t = lane; t < NX * NX; t += WAVE)
          L.P[t] = a.fac(k)[(NV + t / NX) * LDB + NV + t % NX];
      sync();
    }
    return in;
  }
}

// block-chain solve: rhs a.rhs(k) -> gL.u.sol
__device__ __noinline__ void seq_solve(const Agent a) {
  if constexpr (NX > 0) {
    SeqLds& L = gL.u.s;
    const int lane = lane_now();
#pragma unroll 1
    for (int k = 0; k < N; ++k) {
      for (int i = lane; i < NB; i += WAVE) {
        double v = a.rhs(k)[i];
        if (k > 0)
          for (int c = 0; c < NX; ++c) v -= a.cpl(k)[i * NX + c] * L.y[NV + c];
        L.v[i] = v;
      }
      wsync();
      const cdbl* Ai = a.fac(k);
      for (int i = lane; i < NB; i += WAVE) {
        double acc = 0.0;
        for (int j = 0; j < NB; ++j) acc += Ai[i * LDB + j] * L.v[j];
        a.sol(k)[i] = acc;
        L.t[i] = acc;
      }
      wsync();
      for (int i = lane; i < NB; i += WAVE) L.y[i] = L.t[i];
      wsync();
    }
#pragma unroll 1
    for (int k = N - 2; k >= 0; --k) {
      for (int c = lane; c < NX; c += WAVE) {
        double s = 0.0;
        for (int i = 0; i < NB; ++i) s += a.cpl(k + 1)[i * NX + c] * L.y[i];
        L.t[c] = s;
      }
      wsync();
      const cdbl* Ai = a.fac(k);
      for (int i = lane; i < NB; i += WAVE) {
        double u = a.sol(k)[i];
        for (int c = 0; c < NX; ++c) u -= Ai[i * LDB + NV + c] * L.t[c];
        a.sol(k)[i] = u;
        L.v[i] = u;
      }
      wsync();
      for (int i = lane; i < NB; i += WAVE) L.y[i] = L.v[i];
      wsync();
    }
    sync();  // block-chain scratch is dead; sol(.) visible to every lane
    for (int t = lane; t < N * NB; t += WAVE) gL.u.sol[t] = a.sol(t / NB)[t % NB];
    wsync();
  }
}

// ---------------------------------------------------------------------------
// stage-parallel elimination (default path)
// ---------------------------------------------------------------------------
// The KKT matrix, permuted to [all stage interiors | all states], has a block-
// diagonal interior part.  Each stage's interior is Bunch-Kaufman factored by
// G lanes with the two state blocks it touches and the right-hand side appended
// as trailing rows: the elimination leaves the local Schur complement on
// (x_k, x_{k+1}) and the forward-eliminated rhs in those rows.  A backward sweep
// over the trailing rows then yields u0 = A_II^{-1} r_I and Z = A_II^{-1} A_IX,
// so the final solve is u = u0 - Z x: one parallel pass.  The states form a
// block-tridiagonal chain of nx x nx pivots (the only sequential part).
__device__ __forceinline__ int pko(int i) { return (i * (i + 1)) >> 1; }

// local index kinds: 0 primal V, 1 dual (interior rows), 2 x_k, 5 dual mu_k (bordered
// continuity rows), 3 x_{k+1}, 4 border (rhs)
__device__ __forceinline__ int lkind(int i) {
  return i < NV ? 0 : (i < NI ? 1 : (i < LMU ? 2 : (i < LX1 ? 5 : (i < NLOC ? 3 : 4))));
}
__device__ __forceinline__ bool kdual(int kind) { return kind == 1 || kind == 5; }
// local index of constraint row r of a stage, and the row of a local dual index
// (generated tables when continuity rows are bordered, else the identity order)
__device__ __forceinline__ int crow(int r) {
  if constexpr (NMU == 0) return NV + r; else return kCROW[r];
}
__device__ __forceinline__ int lrow(int i) {
  if constexpr (NMU == 0) return i - NV; else return kLROW[i];
}
// index into the stage vector [X0, V, X1] of a primal local index
__device__ __forceinline__ int lnl(int i, int kind) {
  return kind == 0 ? NX + i : (kind == 2 ? i - NI : NX + NV + (i - LX1));
}
// NLP variable index of a primal local index of stage k
__device__ __forceinline__ int lvar(int k, int i, int kind) {
  if (kind == 0) return NX + k * NP + i;
  if (kind == 3) return NX + k * NP + NV + (i - LX1);
  return k == 0 ? (i - NI) : NX + (k - 1) * NP + NV + (i - NI);  // x_k
}
// block-order index ([V, X1, lambda]) of a local index of kind 0, 1, 3, 5
__device__ __forceinline__ int lblk(int i, int kind) {
  return kind == 0 ? i : (kdual(kind) ? NP + lrow(i) : NV + (i - LX1));
}

// diagonal terms (barrier Sigma + delta_w, dual diagonal) and fixed variables
template <int GG, bool COMPACT>
__device__ __forceinline__ void local_diagonal(const Agent a, int k, int g, ldsd* F, const KKTDiag kd,
                                               unsigned long long fm) {
  const wdbl* ws = a.base();
  for (int i = g; i < NLOC; i += GG) {
    const int ki = lkind(i);
    const bool prim = (ki == 0 || ki == 3);
    const bool fixd = (fm >> i) & 1ull;
    const int vi = prim ? lvar(k, i, ki) : 0;
    const int c = kdual(ki) ? k * NG + lrow(i) : 0;
    const double xv = ws[O_X + vi], lo = ws[O_XL + vi], hi = ws[O_XU + vi];
    const double zl = ws[O_ZL + vi], zu = ws[O_ZU + vi];
    const double lbv = ws[O_LB + c], ubv = ws[O_UB + c], sv = ws[O_S + c];
    const double sl = ws[O_SL + c], su = ws[O_SU + c], vl = ws[O_VL + c], vu = ws[O_VU + c];
    const int ii = COMPACT ? i : pko(i) + i;
    if (prim && !fixd) F[ii] += (kd.mode == LSQ) ? 1.0 : sigma_x_v(xv, lo, hi, zl, zu) + kd.dw;
    if (kdual(ki)) F[ii] = -dual_diag_v(cls_of(lbv, ubv, sl, su), sigma_s_v(sv, sl, su, vl, vu), kd);
  }
  wsync();
}

// entry (i, j), i >= j, of stage k's bordered local system gathered from the strided
// derivative arrays (least-squares multiplier system; diagonal terms added afterwards)
__device__ __forceinline__ double generic_entry(const Agent a, int k, int i, int j, unsigned long long fm,
                                                const KKTDiag kd) {
  const wdbl* ws = a.base();
  const int ki = lkind(i), kj = lkind(j);
  const bool pi = (ki == 0 || ki == 2 || ki == 3), pj = (kj == 0 || kj == 2 || kj == 3);
  const bool fi = pi && ((fm >> i) & 1ull), fj = pj && ((fm >> j) & 1ull);
  const bool pp = pi && pj;
  const bool dp = (kdual(ki) && pj) || (kdual(kj) && pi);
  const bool bd = (ki == 4) && (kj != 2 && kj != 4);
  long off = 0, goff = O_GS;
  if (pp) {
    off = O_SDH + ((long)lnl(i, ki) * NL + lnl(j, kj)) * N + k;
  } else if (dp) {
    const int r = lrow(kdual(ki) ? i : j), q = (kdual(ki) ? j : i), kq = (kdual(ki) ? kj : ki);
    off = O_SDJ + ((long)r * NL + lnl(q, kq)) * N + k;
    goff = O_GS + k * NG + r;
  } else if (bd) {
    off = O_RHS + (long)k * NB + lblk(j, kj);
  }
  const double d = (pp || dp) ? a.cold()[off] : ws[off];  // SDH / SDJ: cold part
  const double gsv = ws[goff];
  double v = 0.0;
  if (pp) v = (fi || fj) ? ((i == j && ki == 0) ? 1.0 : 0.0) : (kd.mode == LSQ ? 0.0 : d);
  else if (dp) v = (fi || fj) ? 0.0 : gsv * d;
  else if (bd) v = d;
  return v;
}

// assemble stage k's bordered local system into F, GG lanes: generic gather from the
// strided derivative arrays (least-squares multiplier system); COMPACT: the compact
// image (static path), else the dense packed lower triangle (Bunch-Kaufman path)
template <int GG, bool COMPACT>
__device__ __noinline__ void local_assemble_generic(const Agent a, int k, int g, ldsd* F, const KKTDiag kd) {
  const unsigned long long fm = gL.fixm[k];
#pragma unroll 4
  for (int t = g; t < (COMPACT ? NCPT : PKB); t += GG) {
    int i, j;
    if constexpr (COMPACT) {
      i = kCIJ[t] & 255; j = kCIJ[t] >> 8;
    } else {
      i = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
      if (pko(i + 1) <= t) ++i;
      if (pko(i) > t) --i;
      j = t - pko(i);
    }
    F[t] = generic_entry(a, k, i, j, fm, kd);
  }
  wsync();
  // pass 2: diagonal terms (barrier Sigma + delta_w, dual diagonal)
  local_diagonal<GG, COMPACT>(a, k, g, F, kd, fm);
}

// Newton system of stage k from the compact image the evaluators wrote (stage-minor in
// HBM: the lanes of a round read consecutive stages of one entry), the border from the
// rhs and the diagonal terms the rhs phases wrote: fixed variables (identity row for V, empty row for a state,
// chained as 1) and the diagonal terms the rhs phases precomputed (primal Sigma_x,
// + delta_w here; dual diagonal) are applied on the way.  DENSE: scattered into a zeroed
// dense packed image (Bunch-Kaufman path), else the compact image itself (static path).
template <int GG, bool DENSE>
__device__ MPCX_HOT void local_assemble(const Agent a, int k, int g, ldsd* F, const KKTDiag kd) {
  constexpr int EPC = (NCPT + GG - 1) / GG;  // compact entries per lane
  const unsigned long long fm = gL.fixm[k];
  const wdbl* src = a.lp(k);
  const wdbl* dg = a.dg(k);
  const wdbl* rb = a.rhs(k);
  if constexpr (DENSE) {
    for (int t = g; t < PKB; t += GG) F[t] = 0.0;
    wsync();
  }
  constexpr int CH = EPC < 12 ? EPC : 12;  // entries per lane in flight (loads before the first use)
  const bool anyfix = __ballot(fm != 0ull) != 0ull;  // wave-uniform: some stage of the round has fixed entries
#pragma unroll 1
  for (int e0 = 0; e0 < EPC; e0 += CH) {
    double v[CH], dv[CH];
    int ijv[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int t = g + (e0 + e) * GG;
      // border (rhs) entries from the rhs the rhs phases wrote in block order; x_k has none
      const bool bd = t >= CB && t < CB + NLOC && lkind(t - CB) != 2;
      v[e] = bd ? rb[lblk(t - CB, lkind(t - CB))] : src[(t < NCPT ? t : 0) * N];
      dv[e] = dg[t < NLOC ? t : 0];
      // the entry's (row, column) with the image loads, not under the fixed-entry branch below:
      // kCIJ is a global-memory table, and a load waited for inside a divergent branch drains
      // every older load (r06: one memory round trip per entry of a round holding stage 0)
      ijv[e] = anyfix ? (int)kCIJ[t < NCPT ? t : 0] : 0;
    }
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int t = g + (e0 + e) * GG;
      if (e0 + e >= EPC || t >= NCPT) continue;
      double x = v[e];
      bool fix = false;
      if (fm != 0ull) {
        const int ij = ijv[e], i = ij & 255, j = ij >> 8;
        fix = (((fm >> i) | (fm >> j)) & 1ull) != 0ull;
        if (fix) x = (i == j && lkind(i) == 0) ? 1.0 : 0.0;
      }
      if (t < NLOC) {  // diagonal (t, t)
        const int ki = lkind(t);
        if ((ki == 0 || ki == 3) && !fix) x += dv[e] + kd.dw;
        if (kdual(ki)) x = dv[e];
      }
      F[DENSE ? (int)kCPK[t] : t] = x;
    }
  }
  wsync();
}

// Bunch-Kaufman over the NI interior pivots of one stage (G lanes, packed lower
// storage); the trailing 2*NX state rows and the border row receive the updates
// but never pivot.  bad: singular interior (zero pivot) with coupled stages.
struct BKOut {
  int pos, neg, zero, bad;
};
constexpr int CPL = (RB + G - 1) / G;  // trailing columns per lane (at most RB of them)
__device__ __noinline__ BKOut interior_bk(ldsd* F, ldsi* perm, ldsi* piv, int g) {
  Inertia in{0, 0, 0};
  int bad = 0;
  int k = 0;
#pragma unroll 1
  while (k < NI) {
    double akk = absn(F[pko(k) + k]);
    double lam = -1.0;
    int r = -1;
#pragma unroll
    for (int u = 0; u < (NI + G - 1) / G; ++u) {
      const int i = k + 1 + g + u * G;
      const double t = absn(F[pko(i < NI ? i : k) + k]);
      if (i < NI && t > lam) { lam = t; r = i; }
    }
    gargmax<G>(lam, r);
    if (r < 0) lam = 0.0;
    if (fmax(akk, lam) == 0.0) {
      if constexpr (NX > 0) { bad = 1; break; }
      in.zero++;  // independent stages: a zero column is a zero eigenvalue
      if (g == 0) piv[k] = 1;
      wsync();
      k += 1;
      continue;
    }
    int size = 1, kp = k;
    if (akk < BK_ALPHA * lam) {
      double sg = 0.0;
      for (int j = k + g; j < NI; j += G)
        if (j != r) sg = fmax(sg, absn(F[j < r ? pko(r) + j : pko(j) + r]));
      const double sigma = gmax<G>(sg);
      if (akk * sigma >= BK_ALPHA * lam * lam) {
        kp = k;
      } else if (absn(F[pko(r) + r]) >= BK_ALPHA * sigma) {
        kp = r;
      } else {
        size = 2; kp = r;
      }
    }
    const int p = k + size - 1, q = kp;
    if (q != p) {  // symmetric interchange p <-> q (p < q < NI) in packed storage
      const int op = pko(p), oq = pko(q);
      for (int j = g; j <= RB; j += G) {
        if (j == p) {
          const double t = F[op + p]; F[op + p] = F[oq + q]; F[oq + q] = t;
        } else if (j < p) {
          const double t = F[op + j]; F[op + j] = F[oq + j]; F[oq + j] = t;
        } else if (j < q) {
          const int oj = pko(j);
          const double t = F[oj + p]; F[oj + p] = F[oq + j]; F[oq + j] = t;
        } else if (j > q) {
          const int oj = pko(j);
          const double t = F[oj + p]; F[oj + p] = F[oj + q]; F[oj + q] = t;
        }
      }
      if (g == 0) { const int t = perm[p]; perm[p] = perm[q]; perm[q] = t; }
      wsync();
    }
    // trailing update, column-oriented: lane g owns columns j = k+size+g+u*G and keeps
    // their multipliers in registers; rows in batches of 4 (all reads, then writes);
    // predicated-off writes go to the unused (rhs, rhs) corner instead of branching
    const int DUMMY = pko(RB) + RB;
    if (size == 1) {
      const double d = F[pko(k) + k];
      if (fabs(d) <= ZERO_PIVOT) {
        if constexpr (NX > 0) { bad = 1; break; }
        in.zero++;
      } else if (d > 0) {
        in.pos++;
      } else {
        in.neg++;
      }
      const double rd = 1.0 / d;
      int jj[CPL];
      double lj[CPL];
#pragma unroll
      for (int u = 0; u < CPL; ++u) {
        const int j = k + 1 + g + u * G;
        jj[u] = j;
        lj[u] = (j <= RB) ? F[pko(j <= RB ? j : RB) + k] * rd : 0.0;
      }
#pragma unroll 1
      for (int i0 = k + 1; i0 <= RB; i0 += 4) {
        double aik[4], av[4][CPL];
        int rr[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int ii = (i0 + b <= RB) ? i0 + b : RB;
          rr[b] = pko(ii);
          aik[b] = F[rr[b] + k];
#pragma unroll
          for (int u = 0; u < CPL; ++u) av[b][u] = F[rr[b] + (jj[u] <= ii ? jj[u] : ii)];
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
#pragma unroll
          for (int u = 0; u < CPL; ++u) {
            const bool on = (i0 + b <= RB) && (jj[u] <= i0 + b);
            F[on ? rr[b] + jj[u] : DUMMY] = av[b][u] - aik[b] * lj[u];
          }
        }
      }
      wsync();
#pragma unroll
      for (int u = 0; u < CPL; ++u) F[jj[u] <= RB ? pko(jj[u]) + k : DUMMY] = lj[u];
      if (g == 0) piv[k] = 1;
    } else {
      const int ok = pko(k), ok1 = pko(k + 1);
      const double a11 = F[ok + k], a21 = F[ok1 + k], a22 = F[ok1 + k + 1];
      const double det = a11 * a22 - a21 * a21;
      if (fabs(det) <= ZERO_PIVOT * ZERO_PIVOT) {
        if constexpr (NX > 0) { bad = 1; break; }
        in.zero += 2;
      } else if (det < 0) {
        in.pos++; in.neg++;
      } else if (a11 + a22 > 0) {
        in.pos += 2;
      } else {
        in.neg += 2;
      }
      const double rdet = 1.0 / det;
      int jj[CPL];
      double l1[CPL], l2[CPL];
#pragma unroll
      for (int u = 0; u < CPL; ++u) {
        const int j = k + 2 + g + u * G;
        jj[u] = j;
        const int oj = pko(j <= RB ? j : RB);
        const double aj1 = F[oj + k], aj2 = F[oj + k + 1];
        l1[u] = (j <= RB) ? (aj1 * a22 - aj2 * a21) * rdet : 0.0;
        l2[u] = (j <= RB) ? (aj2 * a11 - aj1 * a21) * rdet : 0.0;
      }
#pragma unroll 1
      for (int i0 = k + 2; i0 <= RB; i0 += 4) {
        double ai1[4], ai2[4], av[4][CPL];
        int rr[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int ii = (i0 + b <= RB) ? i0 + b : RB;
          rr[b] = pko(ii);
          ai1[b] = F[rr[b] + k];
          ai2[b] = F[rr[b] + k + 1];
#pragma unroll
          for (int u = 0; u < CPL; ++u) av[b][u] = F[rr[b] + (jj[u] <= ii ? jj[u] : ii)];
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
#pragma unroll
          for (int u = 0; u < CPL; ++u) {
            const bool on = (i0 + b <= RB) && (jj[u] <= i0 + b);
            F[on ? rr[b] + jj[u] : DUMMY] = av[b][u] - (ai1[b] * l1[u] + ai2[b] * l2[u]);
          }
        }
      }
      wsync();
#pragma unroll
      for (int u = 0; u < CPL; ++u) {
        const int oj = jj[u] <= RB ? pko(jj[u]) : pko(RB);
        F[jj[u] <= RB ? oj + k : DUMMY] = l1[u];
        F[jj[u] <= RB ? oj + k + 1 : DUMMY] = l2[u];
      }
      if (g == 0) { piv[k] = 2; piv[k + 1] = 0; }
    }
    wsync();
    k += size;
  }
  return BKOut{in.pos, in.neg, in.zero, bad};
}

// After interior_bk: back-substitute the trailing rows through L^T, giving
// u0 = L^-T D^-1 z (border row) and Z^T = L^-T L_B^T (state rows).
__device__ __noinline__ void trailing_backsolve(ldsd* F, const ldsi* piv, int g) {
#pragma unroll 1
  for (int m = NI - 1; m > 0; --m) {
    const int skip = (piv[m - 1] == 2) ? m - 1 : -1;
    const int om = pko(m);
    double vt[NTR];
#pragma unroll
    for (int t = 0; t < NTR; ++t) vt[t] = F[pko(NI + t) + m];
    const int DUMMY = pko(RB) + RB;
#pragma unroll
    for (int u = 0; u < (NI + G - 1) / G; ++u) {
      const int i = g + u * G;
      const bool on = i < m && i != skip;
      const int ic = i < m ? i : 0;
      const double lmi = F[om + ic];
      double cur[NTR];
#pragma unroll
      for (int t = 0; t < NTR; ++t) cur[t] = F[pko(NI + t) + ic];
#pragma unroll
      for (int t = 0; t < NTR; ++t) F[on ? pko(NI + t) + ic : DUMMY] = cur[t] - lmi * vt[t];
    }
    wsync();
  }
}

// Chain over the stage boundaries, c_j = [mu_j, x_{j+1}] (NC = NMU + NX): block-tridiagonal
// with the x-part of c_{j-1} coupling to c_j through S10^(j):
//   D_j = S11^(j) + E S00^(j+1) E^T - S10^(j) [D_{j-1}^{-1}]_xx S10^(j)^T
// (E embeds the NX states as the last NX entries of c).  Pivots are BK-factored (indefinite
// when mu is bordered); fixed states are chained as identity rows.
__device__ __forceinline__ const double* s00(int k) { return (const double*)(gL.S + k * SOFF); }
__device__ __forceinline__ const double* s11(int k) { return (const double*)(gL.S + k * SOFF + NXX); }
__device__ __forceinline__ const double* s10(int k) { return (const double*)(gL.S + k * SOFF + NXX + NCC); }

__device__ MPCX_HOT Inertia chain_factor(const Agent a) {
  Lds& L = gL;
  Inertia in{0, 0, 0};
  const int lane = lane_now();
  if constexpr (NX == 1 && NMU == 0) {
    // scalar chain d_j = a_j - b_j / d_{j-1}: lane j gathers its terms in parallel, the
    // recurrence runs on broadcast registers (readlane), fully unrolled
    static_assert(N <= WAVE, "one lane per stage");
    double aj = 0.0, bj = 0.0;
    if (lane < N) {
      const bool fx = (L.fixm[lane] >> LX1) & 1ull;
      aj = fx ? 1.0 : s11(lane)[0] + (lane + 1 < N ? s00(lane + 1)[0] : 0.0);
      if (!fx && lane > 0) { const double t = s10(lane)[0]; bj = t * t; }
    }
    // The pivots d_j = a_j - b_j / d_{j-1} are ratios p_j / p_{j-1} of the three-term recurrence
    // p_j = a_j p_{j-1} - b_j p_{j-2} (leading minors of the chain): lane j forms the prefix
    // product of M_j = [[a_j, -b_j], [1, 0]] by a Hillis-Steele scan inside its row of 16 lanes
    // (DPP row shifts, log2 N steps, each partial product rescaled by a power of two: the ratio
    // of its first column is scale-free), then d_j = P_j[0][0] / P_j[1][0] -- one division per
    // lane instead of N dependent ones.  Near a zero pivot (or on overflow) the serial recurrence
    // runs instead, with its zero-pivot rule (a zero pivot restarts the chain).
    bool serial = true;
    double mine = 0.0;
#ifdef MPCX_CHAIN_SERIAL  // diagnostics (A/B): the serial recurrence only
    if constexpr (false) {
#else
    if constexpr (N <= 16) {
#endif
      double p00 = aj, p01 = -bj, p10 = 1.0, p11 = 0.0;  // lane j: M_j, then M_j ... M_0
      if (lane >= N) { p00 = 1.0; p01 = 0.0; p10 = 0.0; p11 = 1.0; }
#pragma unroll
      for (int sh = 1; sh < N; sh <<= 1) {
        // the partial product ending sh lanes below (row_shr:sh), identity below the row start
        double q00, q01, q10, q11;
        if (sh == 1) { q00 = dpp_f64<0x111>(p00); q01 = dpp_f64<0x111>(p01); q10 = dpp_f64<0x111>(p10); q11 = dpp_f64<0x111>(p11); }
        else if (sh == 2) { q00 = dpp_f64<0x112>(p00); q01 = dpp_f64<0x112>(p01); q10 = dpp_f64<0x112>(p10); q11 = dpp_f64<0x112>(p11); }
        else if (sh == 4) { q00 = dpp_f64<0x114>(p00); q01 = dpp_f64<0x114>(p01); q10 = dpp_f64<0x114>(p10); q11 = dpp_f64<0x114>(p11); }
        else { q00 = dpp_f64<0x118>(p00); q01 = dpp_f64<0x118>(p01); q10 = dpp_f64<0x118>(p10); q11 = dpp_f64<0x118>(p11); }
        if ((lane & 15) >= sh) {
          const double r00 = p00 * q00 + p01 * q10, r01 = p00 * q01 + p01 * q11;
          const double r10 = p10 * q00 + p11 * q10, r11 = p10 * q01 + p11 * q11;
          const double mx = fmax(fmax(fabs(r00), fabs(r01)), fmax(fabs(r10), fabs(r11)));
          const int e = mx > 0.0 && mx < INFINITY ? ilogb(mx) : 0;
          p00 = ldexp(r00, -e); p01 = ldexp(r01, -e); p10 = ldexp(r10, -e); p11 = ldexp(r11, -e);
        }
      }
      const double d = p00 / p10;
      const double r = MPCX_RCP(d);
      // a posteriori: every pivot must satisfy the recurrence with its neighbour's pivot to the
      // rounding of its terms (the minors' products cancel where the chain is nearly singular --
      // restoration phases -- and their errors compound along the scan, unlike the recurrence's)
      const double rprev = dpp_f64<0x111>(r);  // 1 / d_{j-1} (row_shr:1; lane 0 has b_0 = 0)
      const double rec = aj - bj * ((lane & 15) > 0 ? rprev : 0.0);
      const bool ok = lane >= N || (isfin(d) && fabs(d) > 1e-8 * fmax(fabs(aj), 1e-300) && fabs(d) > ZERO_PIVOT &&
                                    fabs(d - rec) <= 1e-12 * (fabs(aj) + fabs(bj * rprev)));
      serial = !__all(ok);
      if (!serial) {
        mine = r;
        const unsigned long long pos = __ballot(lane < N && d > 0.0);
        in.pos = __popcll(pos);
        in.neg = N - in.pos;
      }
    }
    if (serial) {
      double dprev = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const double a = rl_f64(aj, j), b = rl_f64(bj, j);
        const double d = a - b * dprev;
        if (fabs(d) <= ZERO_PIVOT) { in.zero++; dprev = 0.0; }
        else { if (d > 0) in.pos++; else in.neg++; dprev = MPCX_RCP(d); }
        if (lane == j) mine = dprev;
      }
    }
    if (lane < N) L.Dinv[lane] = mine;
  } else if constexpr (NC > 0) {
    constexpr int XO = NMU;  // offset of the states inside c
#pragma unroll 1
    for (int j = 0; j < N; ++j) {
      if (j > 0)  // CW = S10^(j) [D_{j-1}^{-1}]_xx   (NC x NX)
        for (int e = lane; e < NC * NX; e += WAVE) {
          const int r = e / NX, c = e % NX;
          double sacc = 0.0;
          for (int m = 0; m < NX; ++m) sacc += s10(j)[r * NX + m] * L.Dinv[(j - 1) * NCC + (XO + m) * NC + XO + c];
          L.CW[e] = sacc;
        }
      wsync();
      for (int e = lane; e < NCC; e += WAVE) {
        const int r = e / NC, c = e % NC;
        double v = s11(j)[e];
        if (j + 1 < N && r >= XO && c >= XO) v += s00(j + 1)[(r - XO) * NX + (c - XO)];
        if (j > 0)
          for (int m = 0; m < NX; ++m) v -= L.CW[r * NX + m] * s10(j)[c * NX + m];
        const bool fr = r >= XO && ((L.fixm[j] >> (LX1 + r - XO)) & 1ull);
        const bool fc = c >= XO && ((L.fixm[j] >> (LX1 + c - XO)) & 1ull);
        if (fr || fc) v = (r == c) ? 1.0 : 0.0;
        L.C[e] = v;
      }
      wsync();
#ifndef MPCX_CHAIN_BK  // diagnostics: the LDL^T + explicit inverse pair instead of the sweep
      if constexpr (NC * NC <= WAVE) {
        const Inertia bi = bk_sweep<NC, NC>(LDSP(L.C), LDSP(L.Dinv + j * NCC), lane);
        in.pos += bi.pos; in.neg += bi.neg; in.zero += bi.zero;
      } else
#endif
      {
        const Inertia bi = bk_factor<NC, NC>(LDSP(L.C), LDSI(L.cperm), LDSI(L.cpiv), lane);
        in.pos += bi.pos; in.neg += bi.neg; in.zero += bi.zero;
        bk_inverse<NC, NC>(LDSP(L.C), LDSI(L.cperm), LDSI(L.cpiv), LDSP(L.CW), LDSP(L.CY), LDSP(L.Dinv + j * NCC), lane);
      }
    }
  }
  wsync();
  return in;
}

__device__ MPCX_HOT void chain_solve(const Agent a) {
  Lds& L = gL;
  const int lane = lane_now();
  constexpr int ZS = NX + NC;  // zx stride per stage: [x_k | c_k]
  // rhs_j = z[c] of stage j + E z[x_k] of stage j+1
  if constexpr (NX == 1 && NMU == 0) {
    // y_j = c_j - e_j y_{j-1}, x_j = f_j (y_j - g_j x_{j+1}); lane j gathers its terms
    double cj = 0.0, ej = 0.0, fj = 0.0, gj = 0.0;
    if (lane < N) {
      cj = L.zx[lane * 2 + 1] + (lane + 1 < N ? L.zx[(lane + 1) * 2] : 0.0);
      ej = lane > 0 ? s10(lane)[0] * L.Dinv[lane - 1] : 0.0;
      fj = L.Dinv[lane];
      gj = lane + 1 < N ? s10(lane + 1)[0] : 0.0;
    }
    double y = 0.0, yj = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      y = rl_f64(cj, j) - rl_f64(ej, j) * y;
      if (lane == j) yj = y;
    }
    double x = 0.0, xj = 0.0;
#pragma unroll
    for (int j = N - 1; j >= 0; --j) {
      x = rl_f64(fj, j) * (rl_f64(yj, j) - rl_f64(gj, j) * x);
      if (lane == j) xj = x;
    }
    if (lane < N) L.xs[lane] = xj;
  } else if constexpr (NC > 0) {
    constexpr int XO = NMU;
    for (int c = lane; c < NC; c += WAVE)
      L.xs[c] = L.zx[NX + c] + (N > 1 && c >= XO ? L.zx[ZS + (c - XO)] : 0.0);
    wsync();
#pragma unroll 1
    for (int j = 1; j < N; ++j) {
      for (int r = lane; r < NX; r += WAVE) {  // CY = [D_{j-1}^{-1} y_{j-1}]_x
        double sacc = 0.0;
        for (int m = 0; m < NC; ++m) sacc += L.Dinv[(j - 1) * NCC + (XO + r) * NC + m] * L.xs[(j - 1) * NC + m];
        L.CY[r] = sacc;
      }
      wsync();
      for (int r = lane; r < NC; r += WAVE) {
        double v = L.zx[j * ZS + NX + r] + (j + 1 < N && r >= XO ? L.zx[(j + 1) * ZS + (r - XO)] : 0.0);
        for (int m = 0; m < NX; ++m) v -= s10(j)[r * NX + m] * L.CY[m];
        L.xs[j * NC + r] = v;
      }
      wsync();
    }
#pragma unroll 1
    for (int j = N - 1; j >= 0; --j) {
      for (int r = lane; r < NC; r += WAVE) {  // CY = y_j - E S10^(j+1)^T c_{j+1}
        double v = L.xs[j * NC + r];
        if (j + 1 < N && r >= XO)
          for (int m = 0; m < NC; ++m) v -= s10(j + 1)[m * NX + (r - XO)] * L.xs[(j + 1) * NC + m];
        L.CY[r] = v;
      }
      wsync();
      for (int r = lane; r < NC; r += WAVE) {
        double sacc = 0.0;
        for (int m = 0; m < NC; ++m) sacc += L.Dinv[j * NCC + r * NC + m] * L.CY[m];
        L.xs[j * NC + r] = sacc;
      }
      wsync();
    }
  }
  wsync();
}

// Twisted chain (r04): the block-tridiagonal chain eliminated from BOTH ends at once -- forward
// pivots D_j = C_j - S10(j) [D_{j-1}^-1]_xx S10(j)^T for j < CMID, backward pivots
// E_j = C_j - E S10(j+1)^T E_{j+1}^-1 S10(j+1) E^T for j > CMID (E embeds the states), one
// forward and one backward pivot per step swept together (bk_sweep2), and the middle pivot
// M = C_CMID minus both neighbours' contributions last: ceil(N/2) + 1 sequential sweeps instead
// of N.  Another symmetric elimination order of the same matrix, so the same inertia (sum of
// the swept pivots' inertias, Sylvester) and the same solution up to rounding.  Each pivot's
// inverse is swept in place in its Dinv slot.  MPCX_CHAIN_SEQ keeps the one-sided chain (A/B).
#if !defined(MPCX_CHAIN_SEQ) && !defined(MPCX_CHAIN_BK)
constexpr bool CHAIN_TW = NC > 0 && !(NX == 1 && NMU == 0) && NC * NC <= WAVE;
#else
constexpr bool CHAIN_TW = false;
#endif
constexpr int CMID = N / 2;                                        // the middle pivot
constexpr int CSTEPS = CMID > N - 1 - CMID ? CMID : N - 1 - CMID;  // steps before it

__device__ MPCX_HOT Inertia chain_factor_tw(const Agent a) {
  Lds& L = gL;
  Inertia in{0, 0, 0};
  const int lane = lane_now();
  constexpr int XO = NMU;
  constexpr int NCX = NC * NX;
#pragma unroll 1
  for (int s = 0; s <= CSTEPS; ++s) {
    const bool mid = s == CSTEPS;
    const int jf = mid ? CMID : s, jb = N - 1 - s;
    const bool hf = mid || s < CMID;   // a forward pivot (or the middle one) this step
    const bool hb = !mid && jb > CMID;  // a backward pivot this step
    const int jt = mid ? CMID : jb;     // the pivot that takes a backward contribution
    const bool bw = mid ? CMID + 1 < N : hb && jb + 1 < N;
    // CW = S10(jf) [D_{jf-1}^-1]_xx  and  CY = E_{jt+1}^-1 S10(jt+1)   (NC x NX each)
    for (int e = lane; e < 2 * NCX; e += WAVE) {
      const bool sec = e >= NCX;
      const int ee = sec ? e - NCX : e, r = ee / NX, c = ee % NX;
      double sacc = 0.0;
      if (!sec) {
        if (hf && jf > 0)
          for (int m = 0; m < NX; ++m) sacc += s10(jf)[r * NX + m] * L.Dinv[(jf - 1) * NCC + (XO + m) * NC + XO + c];
        L.CW[ee] = sacc;
      } else {
        if (bw)
          for (int m = 0; m < NC; ++m) sacc += L.Dinv[(jt + 1) * NCC + r * NC + m] * s10(jt + 1)[m * NX + c];
        L.CY[ee] = sacc;
      }
    }
    wsync();
    // the pivots, assembled in their Dinv slots
    for (int e = lane; e < 2 * NC * NC; e += WAVE) {
      const bool sec = e >= NC * NC;
      if (sec ? !hb : !hf) continue;
      const int ee = sec ? e - NC * NC : e, r = ee / NC, c = ee % NC;
      const int j = sec ? jb : jf;
      double v = s11(j)[ee];
      if (j + 1 < N && r >= XO && c >= XO) v += s00(j + 1)[(r - XO) * NX + (c - XO)];
      if (!sec && jf > 0)
        for (int m = 0; m < NX; ++m) v -= L.CW[r * NX + m] * s10(jf)[c * NX + m];
      if ((sec || mid) && bw && r >= XO && c >= XO)
        for (int m = 0; m < NC; ++m) v -= s10(jt + 1)[m * NX + (r - XO)] * L.CY[m * NX + (c - XO)];
      const bool fr = r >= XO && ((L.fixm[j] >> (LX1 + r - XO)) & 1ull);
      const bool fc = c >= XO && ((L.fixm[j] >> (LX1 + c - XO)) & 1ull);
      if (fr || fc) v = (r == c) ? 1.0 : 0.0;
      L.Dinv[j * NCC + ee] = v;
    }
    wsync();
    const Inertia bi = bk_sweep2<NC, NC>(LDSP(L.Dinv + jf * NCC), LDSP(L.Dinv + jb * NCC), hb, lane);
    in.pos += bi.pos; in.neg += bi.neg; in.zero += bi.zero;
  }
  wsync();
  return in;
}

// The twisted chain's solve: the rhs eliminated from both ends towards the middle (y_j for
// j < CMID, z_j for j > CMID), the middle block solved, then the back-substitution outwards in
// both directions.  xs holds y / z, then the solution.
__device__ MPCX_HOT void chain_solve_tw(const Agent a) {
  Lds& L = gL;
  const int lane = lane_now();
  constexpr int XO = NMU;
  constexpr int ZS = NX + NC;  // zx stride per stage: [x_k | c_k]
  // rhs of c_j: z[c_j] + E z[x_{j+1}]
  auto rhs = [&](int j, int r) -> double {
    return L.zx[j * ZS + NX + r] + (j + 1 < N && r >= XO ? L.zx[(j + 1) * ZS + (r - XO)] : 0.0);
  };
  for (int e = lane; e < 2 * NC; e += WAVE) {
    const bool sec = e >= NC;
    const int r = sec ? e - NC : e, j = sec ? N - 1 : 0;
    if (sec ? N - 1 > CMID : (CMID > 0 || CSTEPS == 0)) L.xs[j * NC + r] = rhs(j, r);
  }
  wsync();
  // towards the middle: y_j = rhs_j - S10(j) [D_{j-1}^-1 y_{j-1}]_x,
  //                     z_j = rhs_j - E S10(j+1)^T E_{j+1}^-1 z_{j+1}
#pragma unroll 1
  for (int s = 1; s <= CSTEPS; ++s) {
    const bool mid = s == CSTEPS;
    const int jf = mid ? CMID : s, jb = mid ? CMID : N - 1 - s;
    const bool hf = (mid || jf < CMID) && jf > 0, hb = (mid || jb > CMID) && jb + 1 < N;
    for (int e = lane; e < NX + NC; e += WAVE) {
      double sacc = 0.0;
      if (e < NX) {  // CY = [D_{jf-1}^-1 y_{jf-1}]_x
        if (hf)
          for (int m = 0; m < NC; ++m) sacc += L.Dinv[(jf - 1) * NCC + (XO + e) * NC + m] * L.xs[(jf - 1) * NC + m];
        L.CY[e] = sacc;
      } else {  // CW = E_{jb+1}^-1 z_{jb+1}
        const int r = e - NX;
        if (hb)
          for (int m = 0; m < NC; ++m) sacc += L.Dinv[(jb + 1) * NCC + r * NC + m] * L.xs[(jb + 1) * NC + m];
        L.CW[r] = sacc;
      }
    }
    wsync();
    for (int e = lane; e < 2 * NC; e += WAVE) {
      const bool sec = e >= NC;
      const int r = sec ? e - NC : e;
      if (mid && sec) continue;  // the middle block: one update with both terms
      const int j = sec ? jb : jf;
      if (!mid && (sec ? !(jb > CMID) : !(jf < CMID))) continue;
      double v = rhs(j, r);
      if ((!sec || mid) && hf)
        for (int m = 0; m < NX; ++m) v -= s10(jf)[r * NX + m] * L.CY[m];
      if ((sec || mid) && hb && r >= XO)
        for (int m = 0; m < NC; ++m) v -= s10(jb + 1)[m * NX + (r - XO)] * L.CW[m];
      L.xs[j * NC + r] = v;
    }
    wsync();
  }
  // the middle block, then outwards: c_j = D_j^-1 (y_j - E S10(j+1)^T c_{j+1}) for j < CMID,
  //                                  c_j = E_j^-1 (z_j - S10(j) [c_{j-1}]_x)   for j > CMID
#pragma unroll 1
  for (int s = 0; s <= CSTEPS; ++s) {
    const int jf = CMID - s, jb = CMID + s;
    const bool hf = jf >= 0, hb = s > 0 && jb < N;
    for (int e = lane; e < 2 * NC; e += WAVE) {
      const bool sec = e >= NC;
      const int r = sec ? e - NC : e;
      if (sec ? !hb : !hf) continue;
      if (!sec) {
        double v = L.xs[jf * NC + r];
        if (s > 0 && r >= XO)
          for (int m = 0; m < NC; ++m) v -= s10(jf + 1)[m * NX + (r - XO)] * L.xs[(jf + 1) * NC + m];
        L.CY[r] = v;
      } else {
        double v = L.xs[jb * NC + r];
        for (int m = 0; m < NX; ++m) v -= s10(jb)[r * NX + m] * L.xs[(jb - 1) * NC + XO + m];
        L.CW[r] = v;
      }
    }
    wsync();
    for (int e = lane; e < 2 * NC; e += WAVE) {
      const bool sec = e >= NC;
      const int r = sec ? e - NC : e;
      if (sec ? !hb : !hf) continue;
      const int j = sec ? jb : jf;
      const double* src = sec ? (const double*)L.CW : (const double*)L.CY;
      double sacc = 0.0;
      for (int m = 0; m < NC; ++m) sacc += L.Dinv[j * NCC + r * NC + m] * src[m];
      L.xs[j * NC + r] = sacc;
    }
    wsync();
  }
}

// After the interior elimination of stage k (slot lanes g): store its local Schur blocks
// and eliminated rhs (chain input), back-substitute the trailing rows and store the
// back-substitution operators.  A leaf, so factor() keeps almost nothing live across calls.
__device__ __noinline__ void stage_tail(const Agent a, int k, int g, ldsd* F, const ldsi* perm, const ldsi* piv) {
  Lds& L = gL;
  if (NC > 0) {  // local Schur complement on (x_k, c_k), eliminated rhs of those rows
    constexpr int NS = NX * NX + NC * NC + NC * NX;
    for (int e = g; e < NS; e += G) {
      int ri, ci, o;
      if (e < NX * NX) {
        ri = NI + e / NX; ci = NI + e % NX; o = e;
      } else if (e < NX * NX + NC * NC) {
        const int f = e - NX * NX;
        ri = LMU + f / NC; ci = LMU + f % NC; o = NXX + f;
      } else {
        const int f = e - NX * NX - NC * NC;
        ri = LMU + f / NX; ci = NI + f % NX; o = NXX + NCC + f;
      }
      L.S[k * SOFF + o] = (ri >= ci) ? F[pko(ri) + ci] : F[pko(ci) + ri];
    }
    for (int c = g; c < NX + NC; c += G) L.zx[k * (NX + NC) + c] = F[pko(RB) + NI + c];
  }
  trailing_backsolve(F, piv, g);
  // back-substitution operators, column-major [t][p] (the static path stores whole columns)
  for (int p = g; p < NI; p += G) {
#pragma unroll
    for (int t = 0; t < NTR; ++t) a.tr(k)[(t * NI + p) * N] = F[pko(NI + t) + p];
    a.prm(k)[p] = perm[p];
  }
}

#ifdef MPCX_NO_STATIC  // diagnostics: dense Bunch-Kaufman for every stage
#undef MPCX_STATIC_ELIM
#endif
#ifdef MPCX_STATIC_ELIM
// Static sparse elimination of stage k's interior by ONE lane (generated straight-line
// code, runtime/stage_elim.py): writes the Schur blocks, the eliminated rhs and the
// back-substitution operators that interior_bk + stage_tail would.  Eliminates in place
// in the slot's LDS image; returns 1 on a (numerically) singular static pivot, before
// writing any output: the slot is then re-assembled and factored densely.
// The eliminating lane works on a register image of the stage (NCPT doubles) where the register
// budget holds it, so the dependent pivot chain runs on registers instead of LDS round trips (the
// image is scratch: the outputs go to S, ZX and the operators).  Measured on gfx950 (r04,
// profiles/r04/s3, s5): small-fleet builds (one wave per SIMD) spill 12-97 VGPRs with it at NCPT
// 106..202 and none at 67 -> NCPT <= 96 there; fleet builds at one wave per SIMD (MHE, 4 agents
// per CU) 9.76 -> 8.91 ms with the image assembled in registers (scratch 48 -> 176 B/lane); at
// 4 waves per SIMD (C3, 128 VGPRs) it spills 540 B/lane, 2.02 -> 2.43 ms: LDS image there.
#if defined(MPCX_ELIM_NOREG)
constexpr bool ELIM_REG = false;
#elif defined(MPCX_ELIM_FORCE_REG)
constexpr bool ELIM_REG = true;
#elif defined(MPCX_WS_LDS)
constexpr bool ELIM_REG = NCPT <= 96;
#else
constexpr bool ELIM_REG = MIN_WAVES == 1;
#endif

// ... and assembles the Newton systems itself (assemble_reg) unless MPCX_ASM_NOREG (A/B builds)
#ifdef MPCX_ASM_NOREG
constexpr bool ASM_REG = false;
#else
constexpr bool ASM_REG = ELIM_REG;
#endif

template <bool STAGE0, typename FD>
__device__ __forceinline__ int static_body(const Agent a, int k, FD* F, mpcx_elim_ld* S, mpcx_elim_ld* ZX, int* in) {
#ifdef MPCX_STATIC_ELIM0
  // the generated body addresses the workspace with its own pointer types: they must be the
  // workspace's (an HBM-typed pointer into the LDS workspace would be a wild address)
  static_assert(__is_same(mpcx_elim_gd, wdbl) && __is_same(mpcx_elim_gi, wint), "workspace pointer types");
  if constexpr (STAGE0) return gen_stage_elim0(F, S, ZX, (mpcx_elim_gd*)a.tr(k), (mpcx_elim_gi*)a.prm(k), in);
#endif
  return gen_stage_elim(F, S, ZX, (mpcx_elim_gd*)a.tr(k), (mpcx_elim_gi*)a.prm(k), in);
}

// Stage k's compact image assembled by the eliminating lane itself, straight into its registers:
// local_assemble<1, false>'s arithmetic entry by entry (same operations, same order), with no LDS
// image and no wave barrier between assembly and elimination.  The loads are independent (the
// stage-minor image coalesces across the lanes of the round's stages).
__device__ __forceinline__ void assemble_reg(const Agent a, int k, const KKTDiag& kd, double* Fr) {
  const unsigned long long fm = gL.fixm[k];
  const wdbl* src = a.lp(k);
  const wdbl* dg = a.dg(k);
  const wdbl* rb = a.rhs(k);
#pragma unroll
  for (int t = 0; t < NCPT; ++t) {
    // border (rhs) entries from the rhs the rhs phases wrote in block order; x_k has none
    const bool bd = t >= CB && t < CB + NLOC && lkind(t - CB) != 2;
    Fr[t] = bd ? rb[lblk(t - CB, lkind(t - CB))] : src[t * N];
  }
  if (fm != 0ull) {
#pragma unroll
    for (int t = 0; t < NCPT; ++t) {
      const int ij = kCIJ[t], i = ij & 255, j = ij >> 8;
      if ((((fm >> i) | (fm >> j)) & 1ull) != 0ull) Fr[t] = (i == j && lkind(i) == 0) ? 1.0 : 0.0;
    }
  }
#pragma unroll
  for (int t = 0; t < (NLOC < NCPT ? NLOC : NCPT); ++t) {  // diagonal (t, t)
    const int ki = lkind(t);
    const bool fix = ((fm >> t) & 1ull) != 0ull;
    if ((ki == 0 || ki == 3) && !fix) Fr[t] += dg[t] + kd.dw;
    if (kdual(ki)) Fr[t] = dg[t];
  }
}

// kdr: the KKT diagonal terms when the eliminating lane assembles the image itself (ELIM_REG,
// Newton systems), nullptr when the image was assembled into Fl (least-squares system, LDS image)
template <bool STAGE0 = false>
__device__ __forceinline__ int static_stage(const Agent a, int k, ldsd* Fl, const KKTDiag* kdr = nullptr) {
  int in[3];
  asm volatile(";; STATIC_BEGIN");
  mpcx_elim_ld* const S = (mpcx_elim_ld*)LDSP(gL.S + k * SOFF);
  mpcx_elim_ld* const ZX = (mpcx_elim_ld*)LDSP(gL.zx + k * (NX + NC));
  int bad;
  if constexpr (ELIM_REG) {
    double Fr[NCPT];
    if (kdr != nullptr) {
      assemble_reg(a, k, *kdr, Fr);
    } else {
#pragma unroll
      for (int t = 0; t < NCPT; ++t) Fr[t] = Fl[t];
    }
    bad = static_body<STAGE0>(a, k, Fr, S, ZX, in);
  } else {
    bad = static_body<STAGE0>(a, k, (mpcx_elim_ld*)Fl, S, ZX, in);
  }
  asm volatile(";; STATIC_END");
  if (!bad) { atomicAdd(&gL.fin[0], in[0]); atomicAdd(&gL.fin[1], in[1]); }
  return bad;
}
#endif

// q-th set bit of a stage mask (q < popcount)
__device__ __forceinline__ int nth_bit(unsigned long long m, int q) {
  for (int i = 0; i < q; ++i) m &= m - 1ull;
  return __ffsll((long long)m) - 1;
}

// Factor the KKT matrix bordered by the rhs in a.rhs(); returns the inertia.  Only the
// round counter, the inertia sums and the diagonal shifts stay live across the calls.
// Pass 1 (static): SRC compact stage images per round, assembled by GC lanes each and
// eliminated by the generated sparse LDL^T, one lane per stage.  Pass 2 (dense, only
// for the stages pass 1 rejected): SR dense packed images per round, Bunch-Kaufman by
// G lanes each (interior_bk + stage_tail).
__device__ __forceinline__ Inertia factor(const Agent a, const KKTDiag kd) {
  Lds& L = gL;
  SPROF_DECL
  if (lane_now() < 4) L.fin[lane_now()] = 0;  // inertia (pos, neg, zero) and singular flag, summed in LDS
  if (lane_now() < 2) L.dmask[lane_now()] = 0u;
  wsync();
#ifdef MPCX_FORCE_BLOCK_CHAIN  // always take the sequential block chain (diagnostics)
  if constexpr (NX > 0) {
    sync();
    if (!L.sdh_ok && kd.mode != LSQ) {
      eval_hess_impl(a, L.hsig, 1);
      eval_gj_ws(a, a.x(), 1);
      sync();
    }
    if (lane_now() == 0) { L.seq = 1; L.want_sdh = 1; }
    sync();
    return seq_factor(a, kd);
  }
#endif
#ifdef MPCX_STATIC_ELIM
  // register-image builds assemble the Newton systems in the eliminating lane (assemble_reg)
  const bool reg_asm = ASM_REG && kd.mode != LSQ;
#pragma unroll 1
  for (int r = 0; r < CROUNDS; ++r) {
    if (!reg_asm) {
      // stage fastest across the lanes: the stage-minor image reads coalesce over the round
      const int slot = lane_now() % SRC, g = lane_now() / SRC, k = K0 + r * SRC + slot;
      if (g < GC && k < N) {
        ldsd* F = LDSP(L.u.c.F + slot * NCS);
        if (kd.mode == LSQ) local_assemble_generic<GC, true>(a, k, g, F, kd);
        else local_assemble<GC, false>(a, k, g, F, kd);
      }
      wsync();
    }
    SPROF(0);
    {
      const int slot = lane_now(), k = K0 + r * SRC + slot;  // one lane per stage
      if (slot < SRC && k < N && static_stage(a, k, LDSP(L.u.c.F + slot * NCS), reg_asm ? &kd : nullptr)) {
        atomicOr(&L.dmask[k >> 5], 1u << (k & 31));
        atomicAdd(&L.ks.n_dense, 1);
      }
    }
    wsync();
    SPROF(1);
  }
#ifdef MPCX_STATIC_ELIM0
  {  // stage 0 with its own plan (GC lanes assemble into slot 0, one lane eliminates)
    ldsd* F = LDSP(L.u.c.F);
    if (!reg_asm) {
      if (lane_now() < GC) {
        if (kd.mode == LSQ) local_assemble_generic<GC, true>(a, 0, lane_now(), F, kd);
        else local_assemble<GC, false>(a, 0, lane_now(), F, kd);
      }
      wsync();
    }
    if (lane_now() == 0 && static_stage<true>(a, 0, F, reg_asm ? &kd : nullptr)) {
      atomicOr(&L.dmask[0], 1u);
      atomicAdd(&L.ks.n_dense, 1);
    }
    wsync();
    SPROF(1);
  }
#endif
  const unsigned long long dm = ((unsigned long long)L.dmask[1] << 32) | L.dmask[0];
#ifdef MPCX_PROFILE
  if (lane_now() < 2) L.dense_seen[lane_now()] |= L.dmask[lane_now()];
#endif
#else
  const unsigned long long dm = (N == 64) ? ~0ull : ((1ull << N) - 1ull);
#endif
  if (dm != 0ull) {
    const int nd = __popcll(dm);
#pragma unroll 1
    for (int r = 0; r * SR < nd; ++r) {
      {
        const int g = lane_now() % G, slot = lane_now() / G, q = r * SR + slot;
        if (slot < SR && q < nd) {
          const int k = nth_bit(dm, q);
          ldsd* F = LDSP(L.u.p.F + slot * PKS);
          ldsi* perm = LDSI(L.u.p.perm + slot * NI);
          for (int i = g; i < NI; i += G) perm[i] = i;
          if (kd.mode == LSQ) local_assemble_generic<G, false>(a, k, g, F, kd);
          else local_assemble<G, true>(a, k, g, F, kd);
        }
      }
      wsync();
      if (lane_now() / G < SR && r * SR + lane_now() / G < nd) {
        const int g2 = lane_now() % G, slot2 = lane_now() / G;
        const BKOut bo = interior_bk(LDSP(L.u.p.F + slot2 * PKS), LDSI(L.u.p.perm + slot2 * NI),
                                     LDSI(L.u.p.piv + slot2 * NI), g2);
        if (lane_now() % G == 0) {
          atomicAdd(&L.fin[0], bo.pos); atomicAdd(&L.fin[1], bo.neg); atomicAdd(&L.fin[2], bo.zero);
          atomicOr(&L.fin[3], bo.bad);
        }
      }
      wsync();
      SPROF(1);
      if constexpr (NX > 0) {
        if (L.fin[3] != 0) {  // singular stage interior: block chain instead
          sync();
          if (!L.sdh_ok && kd.mode != LSQ) {  // the chain reads the strided Hessians and jacobian
            eval_hess_impl(a, L.hsig, 1);
            eval_gj_ws(a, a.x(), 1);
            sync();
          }
          if (lane_now() == 0) { L.seq = 1; L.want_sdh = 1; }
          sync();
          return seq_factor(a, kd);
        }
      }
      if (lane_now() / G < SR && r * SR + lane_now() / G < nd) {
        const int g = lane_now() % G, slot = lane_now() / G;
        stage_tail(a, nth_bit(dm, r * SR + slot), g, LDSP(L.u.p.F + slot * PKS), LDSI(L.u.p.perm + slot * NI),
                   LDSI(L.u.p.piv + slot * NI));
      }
      wsync();
      SPROF(2);
    }
  }
  Inertia in{L.fin[0], L.fin[1], L.fin[2]};
  if (lane_now() == 0) L.seq = 0;
  if (NC > 0) {
    const Inertia ci = CHAIN_TW ? chain_factor_tw(a) : chain_factor(a);
    in.pos += ci.pos; in.neg += ci.neg; in.zero += ci.zero;
  }
  SPROF(3);
  return in;
}

// stage k of the last factorisation took the dense Bunch-Kaufman path (pivot order in prm)
__device__ __forceinline__ bool stage_was_dense(int k) {
#ifdef MPCX_STATIC_ELIM
  return (gL.dmask[k >> 5] >> (k & 31)) & 1u;
#else
  return true;
#endif
}

// Newton step into gL.u.sol (block order per stage) from the last factorisation.
__device__ MPCX_HOT void solve(const Agent a) {
  Lds& L = gL;
  if (L.seq) { seq_solve(a); return; }
  SPROF_DECL
  const int lane = lane_now();
  if (NC > 0) { if constexpr (CHAIN_TW) chain_solve_tw(a); else chain_solve(a); }
  SPROF(4);
  // u = W [x_k, c_k, 1] per stage interior (operators column-major per stage); the lanes
  // run over all (stage, interior row) pairs, QB rounds of them per batch of operator loads (loaded
  // first, MPCX_PIN: one memory round trip per batch instead of one per round)
  constexpr int QR = (N * NI + WAVE - 1) / WAVE;   // rounds of 64 (stage, row) pairs
  constexpr int QB = cmax(1, cmin(QR, 24 / NTR));  // rounds per batch (<= 24 operator entries per lane)
#pragma unroll 1
  for (int r0 = 0; r0 < QR; r0 += QB) {
    double tv[QB][NTR];
#pragma unroll
    for (int r = 0; r < QB; ++r) {
      const int q = lane + (r0 + r) * WAVE, qq = q < N * NI ? q : 0;
      const int k = qq % N, p = qq / N;  // stage fastest: the stage-minor operator reads coalesce
      const wdbl* t = a.tr(k) + (long)p * N;
#pragma unroll
      for (int c = 0; c < NTR; ++c) tv[r][c] = t[(long)c * NI * N];
    }
#pragma unroll
    for (int r = 0; r < QB; ++r)
#pragma unroll
      for (int c = 0; c < NTR; ++c) MPCX_PIN(tv[r][c]);
#pragma unroll
    for (int r = 0; r < QB; ++r) {
      const int q = lane + (r0 + r) * WAVE;
      if (r0 + r >= QR || q >= N * NI) continue;
      const int k = q % N, p = q / N;
      double u = tv[r][NX + NC];
#pragma unroll
      for (int c = 0; c < NX; ++c) u -= ((k > 0) ? L.xs[(k - 1) * NC + NMU + c] : 0.0) * tv[r][c];
#pragma unroll
      for (int c = 0; c < NC; ++c) u -= L.xs[k * NC + c] * tv[r][NX + c];
      const int o = stage_was_dense(k) ? a.prm(k)[p] : p;  // static stages: identity order
      L.u.sol[k * NB + lblk(o, lkind(o))] = u;
    }
  }
  for (int q = lane; q < N * NC; q += WAVE) {
    const int k = q / NC, li = LMU + q % NC;
    L.u.sol[k * NB + lblk(li, lkind(li))] = L.xs[q];
  }
  wsync();
  SPROF(5);
}

// ---------------------------------------------------------------------------
// vector phases (lane i + 64*slot owns variable / constraint; loads first)
// ---------------------------------------------------------------------------
// push v into [lo + pl, hi - pu] (IPOPT bound_push / bound_frac)
__device__ __forceinline__ double push_into(double v, double lo, double hi, double kp, double kf) {
  const bool hl = isfin(lo), hu = isfin(hi);
  double pl = hl ? kp * fmax(1.0, fabs(lo)) : 0.0;
  double pu = hu ? kp * fmax(1.0, fabs(hi)) : 0.0;
  if (hl && hu) { pl = fmin(pl, kf * (hi - lo)); pu = fmin(pu, kf * (hi - lo)); }
  const double lop = hl ? lo + pl : -INFINITY;
  const double hip = hu ? hi - pu : INFINITY;
  if (hl && hu && lop > hip) return 0.5 * (lo + hi);
  return fmin(fmax(v, lop), hip);
}
__device__ __forceinline__ double relax_lo(double b, double f) { return b - f * fmax(1.0, fabs(b)); }
__device__ __forceinline__ double relax_hi(double b, double f) { return b + f * fmax(1.0, fabs(b)); }

struct Scal {
  double obj_scale, fx;
  int square;  // IPOPT IsSquareProblem: free variables == equality constraints
};

__device__ __noinline__ Scal init_agent(const Agent a, int agent) {
  KArgs* const argp = kargs();
  KArgs& args = *argp;
  const mpcx_options& o = args.opt;
  const int lane = lane_now();
  const gdbl* lbw = (const gdbl*)args.lbw + (long)agent * NW;
  const gdbl* ubw = (const gdbl*)args.ubw + (long)agent * NW;
  const gdbl* wio = (const gdbl*)args.w + (long)agent * NW;
  const gdbl* pin = (const gdbl*)args.p + (long)agent * NPAR;
  for (int t = lane; t < NPAR; t += WAVE) gL.par[t] = pin[t];
  for (long t = lane; t < (long)(2 * NL) * N; t += WAVE) a.base()[O_SDG + t] = 0.0;           // SDG, JTL
  for (long t = lane; t < (long)(NG * NL + NL * NL) * N; t += WAVE) a.cold()[O_SDJ + t] = 0.0;  // SDJ, SDH
  for (long t = lane; t < (long)NCPT * N; t += WAVE) a.base()[O_LP + t] = 0.0;  // structural zeros stay zero
  for (int i = lane; i < NW; i += WAVE) {
    double lo = lbw[i], hi = ubw[i];
    if (lo <= -INF_BOUND) lo = -INFINITY;
    if (hi >= INF_BOUND) hi = INFINITY;
    if (i < NX) hi = lo;  // x_0 is fixed to the initial state (full.py:51-52)
    a.xL()[i] = lo;
    a.xU()[i] = hi;
    a.x()[i] = (lo == hi) ? lo : wio[i];
  }
  if (args.lbg != nullptr) {
    const gdbl* lbg = (const gdbl*)args.lbg + (long)agent * M;
    const gdbl* ubg = (const gdbl*)args.ubg + (long)agent * M;
    for (int c = lane; c < M; c += WAVE) {
      a.lb()[c] = lbg[c];
      a.ub()[c] = ubg[c];
    }
  } else {
    wsync();
    for (int k = lane; k < N; k += WAVE)
      gen_stage_bounds(par_stage(k), par_global(), k * TS, (double*)(a.lb() + k * NG), (double*)(a.ub() + k * NG), 1);
  }
  sync();
  for (int c = lane; c < M; c += WAVE) {
    if (a.lb()[c] <= -INF_BOUND) a.lb()[c] = -INFINITY;
    if (a.ub()[c] >= INF_BOUND) a.ub()[c] = INFINITY;
  }
  for (int c = lane; c < M; c += WAVE) a.gs()[c] = 1.0;
  sync();
  // gradient based scaling at the user starting point
  eval_gj_ws(a, a.x(), 1);
  sync();
  double gmx = 0.0;
  for (int i = NX + lane; i < NW; i += WAVE)
    if (a.xL()[i] != a.xU()[i]) gmx = fmax(gmx, fabs(acc_grad(a, i)));
  gmx = wmax(gmx);
  Scal sc;
  sc.obj_scale = 1.0;
  if (gmx > o.nlp_scaling_max_gradient)
    sc.obj_scale = fmax(o.nlp_scaling_min_value, o.nlp_scaling_max_gradient / gmx);
  for (int c = lane; c < M; c += WAVE) {
    const int k = c / NG, r = c % NG;
    double rm = 0.0;
    for (int j = 0; j < NL; ++j)
      if (a.xL()[k * NP + j] != a.xU()[k * NP + j]) rm = fmax(rm, fabs(a.sdj()[(r * NL + j) * N + k]));
    a.gs()[c] = (rm > o.nlp_scaling_max_gradient) ? fmax(o.nlp_scaling_min_value, o.nlp_scaling_max_gradient / rm) : 1.0;
  }
  // bound relaxation + initial point
  for (int i = lane; i < NW; i += WAVE) {
    double lo = a.xL()[i], hi = a.xU()[i];
    if (i >= NX && lo != hi) {
      if (isfin(lo)) lo = relax_lo(lo, o.bound_relax_factor);
      if (isfin(hi)) hi = relax_hi(hi, o.bound_relax_factor);
      a.xL()[i] = lo;
      a.xU()[i] = hi;
      a.x()[i] = push_into(a.x()[i], lo, hi, o.bound_push, o.bound_frac);
      a.zL()[i] = isfin(lo) ? o.bound_mult_init_val : 0.0;
      a.zU()[i] = isfin(hi) ? o.bound_mult_init_val : 0.0;
    } else {
      a.zL()[i] = 0.0;
      a.zU()[i] = 0.0;
    }
  }
  {  // the variables' bound classes for the hot phases (this lane wrote them above)
    unsigned w = 0u;
    for (int sl = 0; sl < VS; ++sl) {
      const int i = lane + sl * WAVE;
      if (i < NW) {
        const double lo = a.xL()[i], hi = a.xU()[i];
        const unsigned b = ((i >= NX && lo != hi) ? VFREE : 0u) | (isfin(lo) ? VLO : 0u) | (isfin(hi) ? VHI : 0u);
        w |= b << (3 * sl);
      }
    }
    gL.ecls[lane] = w << (2 * CS);  // the rows' classes are added below, once their bounds are final
  }
  sync();
  // fixed-variable masks of the stage-local systems (bounds never change fixedness)
  for (int k = lane; k < N; k += WAVE) {
    unsigned long long m = 0ull;
    for (int i = 0; i < NLOC; ++i) {
      const int ki = lkind(i);
      if (kdual(ki)) continue;
      const int vi = lvar(k, i, ki);
      if (a.xL()[vi] == a.xU()[vi]) m |= 1ull << i;
    }
    gL.fixm[k] = m;
  }
  sc.fx = sc.obj_scale * eval_fg_ws(a, a.x(), a.gv());
  {
    int nfree = 0, neq = 0;
    for (int i = NX + lane; i < NW; i += WAVE) nfree += (a.xL()[i] != a.xU()[i]) ? 1 : 0;
    for (int c = lane; c < M; c += WAVE) neq += (a.lb()[c] == a.ub()[c]) ? 1 : 0;
    sc.square = wsumi(nfree) == wsumi(neq);
  }
  sync();
  for (int c = lane; c < M; c += WAVE) {
    const double gsc = a.gs()[c];
    a.gv()[c] *= gsc;
    const double lo = a.lb()[c], hi = a.ub()[c];
    if (lo == hi) {
      a.sL()[c] = gsc * lo; a.sU()[c] = gsc * hi; a.s()[c] = gsc * lo;
      a.vL()[c] = 0.0; a.vU()[c] = 0.0;
    } else {
      const double sl = isfin(lo) ? relax_lo(gsc * lo, o.bound_relax_factor) : -INFINITY;
      const double su = isfin(hi) ? relax_hi(gsc * hi, o.bound_relax_factor) : INFINITY;
      a.sL()[c] = sl; a.sU()[c] = su;
      a.s()[c] = push_into(a.gv()[c], sl, su, o.bound_push, o.bound_frac);
      a.vL()[c] = isfin(sl) ? o.bound_mult_init_val : 0.0;
      a.vU()[c] = isfin(su) ? o.bound_mult_init_val : 0.0;
    }
    a.lam()[c] = 0.0;
  }
  {  // the rows' classes for the hot phases (this lane wrote its rows' bounds above)
    unsigned w = 0u;
    for (int sl = 0; sl < CS; ++sl) {
      const int c = lane + sl * WAVE;
      if (c < M) w |= (unsigned)cls_of(a.lb()[c], a.ub()[c], a.sL()[c], a.sU()[c]) << (2 * sl);
    }
    gL.ecls[lane] |= w;
  }
  sync();
  eval_gj_ws(a, a.x(), 1);
  sync();
  return sc;
}

// sum |c(x) - s| (scaled) at the current point
__device__ __noinline__ double theta_now(const Agent a) {
  double t = 0.0;
  for (int c = lane_now(); c < M; c += WAVE) {
    const int cl = cls_of(a.lb()[c], a.ub()[c], a.sL()[c], a.sU()[c]);
    const double cv = (cl == 0) ? a.gv()[c] - a.gs()[c] * a.lb()[c] : a.gv()[c] - a.s()[c];
    t += fabs(cv);
  }
  return wsum(t);
}

// dual rows of the rhs (depend on delta_w); ends with the barrier that hands
// the whole rhs to the factorisation lanes
__device__ __noinline__ void rhs_dual(const Agent a, double mu, double dw, double dc) {
  const int lane = lane_now();
  const unsigned cw = cls_word();
#pragma unroll
  for (int sl = 0; sl < CS; ++sl) {
    const int c = lane + sl * WAVE;
    const bool on = c < M;
    const int cc = on ? c : 0;
    const double lbv = a.lb()[cc], slo = a.sL()[cc], sup = a.sU()[cc];
    const double gvv = a.gv()[cc], gsc = a.gs()[cc], sv = a.s()[cc], lm = a.lam()[cc];
    const double vl = a.vL()[cc], vu = a.vU()[cc];
    if (on) {
      const int cl = cls_slot(cw, sl);
      double rr;
      const double rsl = rcp_or0(cl == 1 && isfin(slo), sv - slo), rsu = rcp_or0(cl == 1 && isfin(sup), sup - sv);
      const double rsd = rcp_or0(cl == 1, vl * rsl + vu * rsu + dw);  // 1 / (Sigma_s + delta_w)
      if (cl == 0) {
        rr = -(gvv - gsc * lbv);
      } else {
        rr = -(gvv - sv);
        if (cl == 1) {
          double gphis = 0.0;
          if (isfin(slo)) gphis -= mu * rsl;
          if (isfin(sup)) gphis += mu * rsu;
          rr -= (gphis - lm) * rsd;
        }
      }
      a.rhs(c / NG)[NP + c % NG] = rr;
      a.dg(c / NG)[crow(c % NG)] = (cl == 0) ? -dc : (cl == 2) ? -1.0 : -(rsd + dc);
    }
  }
  sync();
}

// least-squares estimate of the constraint multipliers (IPOPT constr_mult_init_max)
// least-squares estimate of the constraint multipliers (IPOPT constr_mult_init_max): the rhs
// here, the factorisation and solve in the kernel body (inlined there: as part of a called
// phase the factorisation saved every callee-saved VGPR it uses -- MHE 148 per solve), then
// ls_mult_finish
__device__ __noinline__ void ls_mult_rhs(const Agent a, double obj_scale) {
  const int lane = lane_now();
  for (int i = NX + lane; i < NW; i += WAVE) {
    const double r = (a.xL()[i] == a.xU()[i]) ? 0.0 : -(obj_scale * acc_grad(a, i) - a.zL()[i] + a.zU()[i]);
    a.rhs((i - NX) / NP)[(i - NX) % NP] = r;
  }
  for (int c = lane; c < M; c += WAVE) {
    const int cl = cls_of(a.lb()[c], a.ub()[c], a.sL()[c], a.sU()[c]);
    a.rhs(c / NG)[NP + c % NG] = (cl == 1) ? a.vL()[c] - a.vU()[c] : 0.0;
  }
  sync();
}
__device__ __noinline__ void ls_mult_finish(const Agent a, const double constr_mult_init_max) {
  const int lane = lane_now();
  double lmax = 0.0;
  for (int c = lane; c < M; c += WAVE) lmax = fmax(lmax, fabs(gL.u.sol[(c / NG) * NB + NP + c % NG]));
  lmax = wmax(lmax);
  if (lmax <= constr_mult_init_max) {
    for (int c = lane; c < M; c += WAVE) a.lam()[c] = gL.u.sol[(c / NG) * NB + NP + c % NG];
    sync();
    eval_gj_ws(a, a.x(), 0);  // (J~^T lambda) of the new multipliers
  }
  sync();
}


// full step from the Newton solution (LDS) + fraction-to-the-boundary step
// sizes + constraint violation and barrier at the current point
// running minimum of step-size ratios num / den (num >= 0, den > 0) kept as the pair: one
// division per lane at the end instead of one per candidate; the quotient taken is the one the
// per-candidate division gives for the minimising candidate (rounding is monotone)
#ifndef MPCX_RATIO_FMIN
struct RatioMin {
  double n = 1.0, d = 1.0;  // the default step size 1
  __device__ __forceinline__ void take(double num, double den) {
    const double l = num * d, r = n * den;
    // the cross products leave the normal range only for extreme slacks / step components (the
    // ill-conditioned restoration cases): there the quotients are compared, as fmin(num / den) did
    // (a branch of its own, kept from being if-converted by the empty volatile asm: the divisions
    // run only when a lane needs them)
    const bool exact = __builtin_isnormal(l) && __builtin_isnormal(r);  // v_cmp_class each
    bool lt;
    if (__builtin_expect(exact, 1)) {
      lt = l < r;
    } else {
      asm volatile("");
      lt = num / den < n / d;
    }
    if (lt) { n = num; d = den; }
  }
  __device__ __forceinline__ double value() const { return n / d; }
};
#else  // diagnostics (A/B): one division per candidate
struct RatioMin {
  double v = 1.0;
  __device__ __forceinline__ void take(double num, double den) { v = fmin(v, num / den); }
  __device__ __forceinline__ double value() const { return v; }
};
#endif

// Sum of logs of a lane's slacks as ONE log: the mantissas multiplied (each in [0.5, 1), a lane
// takes at most a few dozen: no underflow), the exponents summed, log(prod) + e ln 2 at the end
// (r05: the trial point's barrier took a log -- ~35 dependent instructions -- per slack)
struct LogSum {
  double m = 1.0;
  int e = 0;
  __device__ __forceinline__ void add(double s) {
    int k;
    const double f = frexp(s, &k);
    m *= s < 0 ? __builtin_nan("") : f;   // a negative slack: NaN like its log (0 -> -inf, as log)
    e += k;
  }
};
constexpr double LN2 = 0.6931471805599453;

// full step from the Newton solution (LDS) + fraction-to-the-boundary step sizes + constraint
// violation at the current point; the barrier sum too unless the caller passes the cached one
// (bar_cached: the current point is the last accepted trial point, whose logs the line search
// summed -- the logs were a fifth of this phase's instructions)
__device__ MPCX_HOT StepInfo recover_step(const Agent a, double mu, double tau, double dw, double obj_scale,
                                          int bar_cached) {
  const int lane = lane_now();
  RatioMin ra, rz;
  LogSum lb;
  double gphid = 0.0, theta = 0.0;
  const unsigned vw = vcls_word(), cw = cls_word();
  // every operand of the phase loaded first, in one batch (MPCX_PIN: one memory round trip)
  double lo[VS], hi[VS], xv[VS], zl[VS], zu[VS], gr[VS], sx[VS];
#pragma unroll
  for (int sl = 0; sl < VS; ++sl) {
    const int i = lane + sl * WAVE;
    const int ii = (i >= NX && i < NW) ? i : NX;
    lo[sl] = a.xL()[ii]; hi[sl] = a.xU()[ii]; xv[sl] = a.x()[ii]; zl[sl] = a.zL()[ii]; zu[sl] = a.zU()[ii];
    gr[sl] = acc_grad(a, ii);
    sx[sl] = gL.u.sol[((ii - NX) / NP) * NB + (ii - NX) % NP];
  }
#pragma unroll
  for (int sl = 0; sl < VS; ++sl) { MPCX_PIN(lo[sl]); MPCX_PIN(hi[sl]); MPCX_PIN(xv[sl]); MPCX_PIN(zl[sl]); MPCX_PIN(zu[sl]); MPCX_PIN(gr[sl]); }
#pragma unroll
  for (int sl = 0; sl < VS; ++sl) {
    const int i = lane + sl * WAVE;
    if (i >= NW) continue;
    const unsigned vb = vcls_slot(vw, sl);
    const bool free_ = (vb & VFREE) != 0u;
    const double d = free_ ? sx[sl] : 0.0;
    a.dx()[i] = d;
    if (!free_) continue;
    double gphi = obj_scale * gr[sl];
    if (vb & VLO) {
      const double s_l = xv[sl] - lo[sl], rl = MPCX_RCP(s_l);
      gphi -= mu * rl;
      if (d < 0) ra.take(tau * s_l, -d);
      const double dz = mu * rl - zl[sl] - (zl[sl] * rl) * d;
      if (dz < 0) rz.take(tau * zl[sl], -dz);
      if (!bar_cached) lb.add(s_l);
    }
    if (vb & VHI) {
      const double s_u = hi[sl] - xv[sl], ru = MPCX_RCP(s_u);
      gphi += mu * ru;
      if (d > 0) ra.take(tau * s_u, d);
      const double dz = mu * ru - zu[sl] + (zu[sl] * ru) * d;
      if (dz < 0) rz.take(tau * zu[sl], -dz);
      if (!bar_cached) lb.add(s_u);
    }
    gphid += gphi * d;
  }
  // the constraints' operands: a second batch (both at once would need more registers than a leaf
  // phase has without saving callee-saved ones: 22 scratch saves and restores per call, C3 +4 %, r06/s5)
  double lbv[CS], slo[CS], sup[CS], sv[CS], lm[CS], vl[CS], vu[CS], gvv[CS], gsc[CS], dlam[CS];
#pragma unroll
  for (int sl = 0; sl < CS; ++sl) {
    const int c = lane + sl * WAVE;
    const int cc = c < M ? c : 0;
    lbv[sl] = a.lb()[cc]; slo[sl] = a.sL()[cc]; sup[sl] = a.sU()[cc]; sv[sl] = a.s()[cc]; lm[sl] = a.lam()[cc];
    vl[sl] = a.vL()[cc]; vu[sl] = a.vU()[cc]; gvv[sl] = a.gv()[cc]; gsc[sl] = a.gs()[cc];
    dlam[sl] = gL.u.sol[(cc / NG) * NB + NP + cc % NG];
  }
#pragma unroll
  for (int sl = 0; sl < CS; ++sl) {
    MPCX_PIN(lbv[sl]); MPCX_PIN(slo[sl]); MPCX_PIN(sup[sl]); MPCX_PIN(sv[sl]); MPCX_PIN(lm[sl]);
    MPCX_PIN(vl[sl]); MPCX_PIN(vu[sl]); MPCX_PIN(gvv[sl]); MPCX_PIN(gsc[sl]);
  }
#pragma unroll
  for (int sl = 0; sl < CS; ++sl) {
    const int c = lane + sl * WAVE;
    if (c >= M) continue;
    a.dl()[c] = dlam[sl];
    const int cl = cls_slot(cw, sl);
    theta += fabs((cl == 0) ? gvv[sl] - gsc[sl] * lbv[sl] : gvv[sl] - sv[sl]);
    double dsv = 0.0;
    if (cl == 1) {
      const double rsl = rcp_or0(isfin(slo[sl]), sv[sl] - slo[sl]), rsu = rcp_or0(isfin(sup[sl]), sup[sl] - sv[sl]);
      double gphis = 0.0;
      if (isfin(slo[sl])) gphis -= mu * rsl;
      if (isfin(sup[sl])) gphis += mu * rsu;
      const double rs = gphis - lm[sl];
      dsv = (dlam[sl] - rs) * MPCX_RCP(vl[sl] * rsl + vu[sl] * rsu + dw);
      gphid += (rs + lm[sl]) * dsv;
      if (isfin(slo[sl])) {
        const double s_l = sv[sl] - slo[sl];
        if (dsv < 0) ra.take(tau * s_l, -dsv);
        const double dv = mu * rsl - vl[sl] - (vl[sl] * rsl) * dsv;
        if (dv < 0) rz.take(tau * vl[sl], -dv);
        if (!bar_cached) lb.add(s_l);
      }
      if (isfin(sup[sl])) {
        const double s_u = sup[sl] - sv[sl];
        if (dsv > 0) ra.take(tau * s_u, dsv);
        const double dv = mu * rsu - vu[sl] + (vu[sl] * rsu) * dsv;
        if (dv < 0) rz.take(tau * vu[sl], -dv);
        if (!bar_cached) lb.add(s_u);
      }
    }
    a.ds()[c] = dsv;
  }
  StepInfo st;
  st.amax = wmin(ra.value());
  st.az = wmin(rz.value());
  st.gphid = wsum(gphid);
  st.theta = wsum(theta);
  st.barrier = bar_cached ? gL.ks.bar_val : wsum(log(lb.m) + lb.e * LN2);
  return st;
}

__device__ __noinline__ bool spill_dominates(double th, double ph);  // the filter's spill list (below)

struct LSOpt {  // line-search options by value (registers, not kernarg loads)
  double alpha_min_frac, gamma_theta, gamma_phi, delta, s_theta, s_phi, eta_phi;
};

// pow / log out of line: inlined into a loop that also calls a phase function, their
// polynomial constants are hoisted into VGPRs that live across the call (scratch spills)
__device__ MPCX_HOT double pow_ool(double x, double y) { return pow(x, y); }
__device__ MPCX_HOT double log_ool(double x) { return log(x); }

// filter line search from the recovered step (gL.ks.st) into gL.ks.ls; trial points live
// in LDS (xt, scaled gt).  The search state is kept in LDS too and nothing vector-sized
// stays in registers across the evaluation call (a non-leaf function saves every
// callee-saved VGPR it uses to scratch): the x-part of the barrier is summed while the
// trial point is written, the constraint part is re-read after the call.
__device__ MPCX_HOT void line_search(const Agent a) {
  KArgs* const argp = kargs();
  KState& K = gL.ks;
  {
    KArgs& ka = *argp;
    const double gphid = K.st.gphid, theta = K.st.theta;
    // the switching condition's powers are loop invariant (only alpha changes between trials)
    K.sw_l = gphid < 0 ? pow_ool(-gphid, ka.opt.s_phi) : 0.0;
    K.sw_r = gphid < 0 ? ka.opt.delta * pow_ool(theta, ka.opt.s_theta) : 0.0;
    double amin;
    if (gphid < 0 && theta <= K.theta_min)
      amin = ka.opt.alpha_min_frac * fmin(fmin(ka.opt.gamma_theta, ka.opt.gamma_phi * theta / (-gphid)),
                                     K.sw_r / K.sw_l);
    else if (gphid < 0)
      amin = ka.opt.alpha_min_frac * fmin(ka.opt.gamma_theta, ka.opt.gamma_phi * theta / (-gphid));
    else
      amin = ka.opt.alpha_min_frac * ka.opt.gamma_theta;
    if (!(amin > 0.0)) amin = ka.opt.alpha_min_frac * ka.opt.gamma_theta;  // NaN guard
    K.amin = amin;
    // soft restoration step (K.lsmode == 1): ONE trial at the full fraction-to-the-boundary
    // step of primal and dual variables, tested at alpha = 0 (no switching condition)
    K.ls.alpha = K.lsmode ? fmin(K.st.amax, K.st.az) : K.st.amax;
    K.ls.accepted = 0;
    K.ls.ftype = 0;
    K.ls.trials = 0;
    K.ls.tr = Trial{0.0, 0.0, 0.0, 0.0};
    K.ls.bar = 0.0;
    TRACE_LS_HEAD(argp);
  }
#pragma unroll 1
  for (int ls = 0; ls < 64; ++ls) {
    {
      const int lane = lane_now();
      const double alpha = K.ls.alpha;
      LogSum bx;
      const unsigned vw = vcls_word();
      double lo[VS], hi[VS], xv[VS], dx[VS];  // loaded first, one batch (MPCX_PIN)
#pragma unroll
      for (int sl = 0; sl < VS; ++sl) {
        const int i = lane + sl * WAVE, ii = i < NW ? i : 0;
        lo[sl] = a.xL()[ii]; hi[sl] = a.xU()[ii]; xv[sl] = a.x()[ii]; dx[sl] = a.dx()[ii];
      }
#pragma unroll
      for (int sl = 0; sl < VS; ++sl) { MPCX_PIN(lo[sl]); MPCX_PIN(hi[sl]); MPCX_PIN(xv[sl]); MPCX_PIN(dx[sl]); }
#pragma unroll
      for (int sl = 0; sl < VS; ++sl) {
        const int i = lane + sl * WAVE;
        if (i < NW) {
          const unsigned vb = vcls_slot(vw, sl);
          const double xt = xv[sl] + alpha * dx[sl];
          gL.u.t.xt[i] = xt;
          if (vb & VFREE) {
            if (vb & VLO) bx.add(xt - lo[sl]);
            if (vb & VHI) bx.add(hi[sl] - xt);
          }
        }
      }
      K.barx = wsum(log_ool(bx.m) + bx.e * LN2);
    }
    wsync();
    {
      const double f = eval_fg_lds(a);
      K.ls.tr.f = K.obj_scale * f;
    }
    wsync();
    const int lane = lane_now();
    const double alpha = K.ls.alpha;
    double th = 0.0;
    LogSum bs;
    const unsigned cw = cls_word();
    double gsv[CS], lbv[CS], slv[CS], suv[CS], sv[CS], dsv[CS];  // loaded first, one batch (MPCX_PIN)
#pragma unroll
    for (int sl = 0; sl < CS; ++sl) {
      const int c = lane + sl * WAVE, cc = c < M ? c : 0;
      gsv[sl] = a.gs()[cc]; lbv[sl] = a.lb()[cc]; slv[sl] = a.sL()[cc]; suv[sl] = a.sU()[cc];
      sv[sl] = a.s()[cc]; dsv[sl] = a.ds()[cc];
    }
#pragma unroll
    for (int sl = 0; sl < CS; ++sl) {
      MPCX_PIN(gsv[sl]); MPCX_PIN(lbv[sl]); MPCX_PIN(slv[sl]); MPCX_PIN(suv[sl]); MPCX_PIN(sv[sl]); MPCX_PIN(dsv[sl]);
    }
#pragma unroll
    for (int sl = 0; sl < CS; ++sl) {
      const int c = lane + sl * WAVE;
      if (c < M) {
        const int cl = cls_slot(cw, sl);
        const double gt = gL.u.t.gt[c] * gsv[sl];
        gL.u.t.gt[c] = gt;
        const double st = sv[sl] + alpha * dsv[sl];
        th += fabs(cl == 0 ? gt - gsv[sl] * lbv[sl] : gt - st);
        if (cl == 1) {
          if (isfin(slv[sl])) bs.add(st - slv[sl]);
          if (isfin(suv[sl])) bs.add(suv[sl] - st);
        }
      }
    }
    const double bar = log_ool(bs.m) + bs.e * LN2;
    KArgs& ka = *argp;
    const double mu = K.mu, theta = K.st.theta, gphid = K.st.gphid;
    const double phi = K.fx - mu * K.st.barrier;
    Trial tr = K.ls.tr;
    tr.theta = wsum(th);
    const double trial_bar = K.barx + wsum(bar);
    tr.phi = tr.f - mu * trial_bar;
    K.ls.tr = tr;
    K.ls.bar = trial_bar;
    K.ls.trials += 1;
    // a trial whose barrier function is not finite (a slack rounded to 0: phi = +inf) is cut back like
    // an evaluation error (IPOPT BacktrackingLineSearch; oracle/ipm.py rejects it) -- the theta-reduction
    // branch below would otherwise take it and the next iterate's barrier terms are inf / NaN
    bool okt = (tr.theta <= K.theta_max) && isfin(tr.phi);
    {  // filter test, one entry per lane (MAXF <= 64): one LDS read instead of nfilt in sequence
      const int j = lane_now();
      const bool dom = j < K.nfilt && tr.theta >= gL.fth[j < MAXF ? j : 0] && tr.phi >= gL.fph[j < MAXF ? j : 0];
      if (__any(dom)) okt = false;
      if (okt && K.nsp[K.resto] > 0 && spill_dominates(tr.theta, tr.phi)) okt = false;  // older entries
    }
    const bool okf = okt;
    (void)okf;
    bool ftype = false;
    if (okt) {
      const bool switching = !K.lsmode && gphid < 0 && alpha * K.sw_l > K.sw_r;
      if (theta <= K.theta_min && switching) {
        okt = tr.phi <= phi + ka.opt.eta_phi * alpha * gphid;
        ftype = true;
      } else {
        okt = tr.theta <= (1.0 - ka.opt.gamma_theta) * theta || tr.phi <= phi - ka.opt.gamma_phi * theta;
        ftype = false;
      }
    }
    K.ls.ftype = ftype;
    TRACE_LS_TRIAL(argp, alpha, tr, okf, okt, ftype);
    if (okt) { K.ls.accepted = 1; break; }
    if (K.lsmode || alpha * 0.5 < K.amin) break;
    K.ls.alpha = alpha * 0.5;
  }
  wsync();
}

// take the last trial point (xt, gt in LDS) and the multiplier steps
__device__ MPCX_HOT void accept_step(const Agent a, const double kappa_sigma, double mu, double alpha, double az) {
  const int lane = lane_now();
  const double ksm = kappa_sigma * mu, mks = mu * MPCX_RCP(kappa_sigma);  // the kappa_sigma safeguard's bounds x s
  const unsigned vw = vcls_word(), cw = cls_word();
  // every operand loaded first, one batch (MPCX_PIN), then the updates and stores
  double lo[VS], hi[VS], xold[VS], dx[VS], zl[VS], zu[VS], xn[VS];
#pragma unroll
  for (int sl = 0; sl < VS; ++sl) {
    const int i = lane + sl * WAVE;
    const int ii = (i >= NX && i < NW) ? i : NX;
    lo[sl] = a.xL()[ii]; hi[sl] = a.xU()[ii]; xold[sl] = a.x()[ii]; dx[sl] = a.dx()[ii];
    zl[sl] = a.zL()[ii]; zu[sl] = a.zU()[ii];
    xn[sl] = gL.u.t.xt[ii];
  }
#pragma unroll
  for (int sl = 0; sl < VS; ++sl) {
    MPCX_PIN(lo[sl]); MPCX_PIN(hi[sl]); MPCX_PIN(xold[sl]); MPCX_PIN(dx[sl]); MPCX_PIN(zl[sl]); MPCX_PIN(zu[sl]);
  }
#pragma unroll
  for (int sl = 0; sl < VS; ++sl) {
    const int i = lane + sl * WAVE;
    const unsigned vb = vcls_slot(vw, sl);
    if (!(vb & VFREE)) continue;  // VFREE: NX <= i < NW, lo != hi
    a.x()[i] = xn[sl];
    if (vb & VLO) {
      const double r0 = MPCX_RCP(xold[sl] - lo[sl]);
      const double dz = mu * r0 - zl[sl] - (zl[sl] * r0) * dx[sl];
      const double zn = zl[sl] + az * dz, rn = MPCX_RCP(xn[sl] - lo[sl]);
      a.zL()[i] = fmax(fmin(zn, ksm * rn), mks * rn);
    }
    if (vb & VHI) {
      const double r0 = MPCX_RCP(hi[sl] - xold[sl]);
      const double dz = mu * r0 - zu[sl] + (zu[sl] * r0) * dx[sl];
      const double zn = zu[sl] + az * dz, rn = MPCX_RCP(hi[sl] - xn[sl]);
      a.zU()[i] = fmax(fmin(zn, ksm * rn), mks * rn);
    }
  }
  // the constraints' operands: a second batch (register budget of a leaf phase, see recover_step)
  double slo[CS], sup[CS], lm[CS], dl[CS], sold[CS], dsv[CS], vl[CS], vu[CS], gt[CS];
#pragma unroll
  for (int sl = 0; sl < CS; ++sl) {
    const int c = lane + sl * WAVE;
    const int cc = c < M ? c : 0;
    slo[sl] = a.sL()[cc]; sup[sl] = a.sU()[cc]; lm[sl] = a.lam()[cc]; dl[sl] = a.dl()[cc]; sold[sl] = a.s()[cc];
    dsv[sl] = a.ds()[cc]; vl[sl] = a.vL()[cc]; vu[sl] = a.vU()[cc];
    gt[sl] = gL.u.t.gt[cc];
  }
#pragma unroll
  for (int sl = 0; sl < CS; ++sl) {
    MPCX_PIN(slo[sl]); MPCX_PIN(sup[sl]); MPCX_PIN(lm[sl]); MPCX_PIN(dl[sl]); MPCX_PIN(sold[sl]);
    MPCX_PIN(dsv[sl]); MPCX_PIN(vl[sl]); MPCX_PIN(vu[sl]);
  }
#pragma unroll
  for (int sl = 0; sl < CS; ++sl) {
    const int c = lane + sl * WAVE;
    if (c >= M) continue;
    a.lam()[c] = lm[sl] + alpha * dl[sl];
    a.gv()[c] = gt[sl];
    const double sn = sold[sl] + alpha * dsv[sl];
    a.s()[c] = sn;
    if (cls_slot(cw, sl) != 1) continue;
    if (isfin(slo[sl])) {
      const double r0 = MPCX_RCP(sold[sl] - slo[sl]);
      const double dv = mu * r0 - vl[sl] - (vl[sl] * r0) * dsv[sl];
      const double vn = vl[sl] + az * dv, rn = MPCX_RCP(sn - slo[sl]);
      a.vL()[c] = fmax(fmin(vn, ksm * rn), mks * rn);
    }
    if (isfin(sup[sl])) {
      const double r0 = MPCX_RCP(sup[sl] - sold[sl]);
      const double dv = mu * r0 - vu[sl] + (vu[sl] * r0) * dsv[sl];
      const double vn = vu[sl] + az * dv, rn = MPCX_RCP(sup[sl] - sn);
      a.vU()[c] = fmax(fmin(vn, ksm * rn), mks * rn);
    }
  }
}

// IPOPT OptimalityErrorConvergenceCheck::CurrentIsAcceptable: the objective-change test
// compares the (scaled) objective of the last two iterations at which it was called
// (initially -1e50, so the first call never passes a finite acceptable_obj_change_tol)
__device__ __forceinline__ bool current_is_acceptable(Acceptable& ac, const OptErr& e, double err0, double fx,
                                                      int it, double obj_scale, int square,
                                                      const mpcx_options& o) {
  if (it != ac.last_it) { ac.last_f = ac.curr_f; ac.curr_f = fx; ac.last_it = it; }
  if (square) return err0 <= o.acceptable_tol && e.viol_u <= o.acceptable_constr_viol_tol;
  return err0 <= o.acceptable_tol && e.dual_u <= o.acceptable_dual_inf_tol &&
         e.viol_u <= o.acceptable_constr_viol_tol && e.compl_at(0.0) / obj_scale <= o.acceptable_compl_inf_tol &&
         fabs(ac.curr_f - ac.last_f) / fmax(1.0, fabs(ac.curr_f)) <= o.acceptable_obj_change_tol;
}


// Top of an IPM iteration in ONE pass over the variables and constraints: IPOPT's scaled
// optimality error, the termination tests (tol, acceptable level, max_iter), the monotone
// barrier update, then the Newton rhs and the KKT diagonal terms at the new mu for
// delta_w = delta_c = 0 (what rhs_dual recomputes for an inertia correction).  The
// operands are loaded once and stay in registers across the wave reductions (no calls),
// instead of being streamed again by separate rhs phases.  Returns 1 when the solve stops
// (K.status set), 0 with the rhs handed to the factorisation lanes (barrier).
__device__ __attribute__((always_inline)) int iter_head(const Agent a) {
  KArgs* const argp = kargs();
  KArgs& ka = *argp;
  KState& K = gL.ks;
  const int lane = lane_now();
  const double obj_scale = K.obj_scale;
  // what the rhs needs is reduced to 3 values per slot while the error terms are summed, the
  // rhs being affine in mu: primal r = r0 + mu r1 (r0 = -(obj_scale grad + J~^T lam),
  // r1 = 1/(x - lo) - 1/(hi - x)) and Sigma_x; dual (inequality rows) rr = q0 - mu q1
  // (q0 = -(c - s) + lam / Sigma_s, q1 = (1/(sU - s) - 1/(s - sL)) / Sigma_s) and the dual
  // diagonal; equality / free rows: rr = q0
  SPROF_DECL
  double pr0[VS], pr1[VS], psx[VS];
  double dq0[CS], dq1[CS], ddg[CS];
  {
    double dmax = 0.0, dmax_u = 0.0, pmax = 0.0, vmax_u = 0.0, pmx = -INFINITY, pmn = INFINITY;
    double lsum = 0.0, zsum = 0.0;
    int nz = 0;
    const unsigned vw = vcls_word(), cw = cls_word();
    // every operand loaded first, one batch (MPCX_PIN: one memory round trip instead of one per slot)
    double lo_[VS], hi_[VS], xv_[VS], zl_[VS], zu_[VS], gr_[VS], jt_[VS];
#pragma unroll
    for (int sl = 0; sl < VS; ++sl) {
      const int i = lane + sl * WAVE;
      const int ii = (i >= NX && i < NW) ? i : NX;
      lo_[sl] = a.xL()[ii]; hi_[sl] = a.xU()[ii]; xv_[sl] = a.x()[ii]; zl_[sl] = a.zL()[ii]; zu_[sl] = a.zU()[ii];
      gr_[sl] = acc_grad(a, ii); jt_[sl] = acc_jtl(a, ii);
    }
    double lb_[CS], sl_[CS], su_[CS], gs_[CS], lm_[CS], gv_[CS], sv_[CS], vl_[CS], vu_[CS];
#pragma unroll
    for (int sl = 0; sl < CS; ++sl) {
      const int c = lane + sl * WAVE;
      const int cc = c < M ? c : 0;
      lb_[sl] = a.lb()[cc]; sl_[sl] = a.sL()[cc]; su_[sl] = a.sU()[cc]; gs_[sl] = a.gs()[cc]; lm_[sl] = a.lam()[cc];
      gv_[sl] = a.gv()[cc]; sv_[sl] = a.s()[cc]; vl_[sl] = a.vL()[cc]; vu_[sl] = a.vU()[cc];
    }
#pragma unroll
    for (int sl = 0; sl < VS; ++sl) {
      MPCX_PIN_HEAD(lo_[sl]); MPCX_PIN_HEAD(hi_[sl]); MPCX_PIN_HEAD(xv_[sl]); MPCX_PIN_HEAD(zl_[sl]); MPCX_PIN_HEAD(zu_[sl]);
      MPCX_PIN_HEAD(gr_[sl]); MPCX_PIN_HEAD(jt_[sl]);
    }
#pragma unroll
    for (int sl = 0; sl < CS; ++sl) {
      MPCX_PIN_HEAD(lb_[sl]); MPCX_PIN_HEAD(sl_[sl]); MPCX_PIN_HEAD(su_[sl]); MPCX_PIN_HEAD(gs_[sl]); MPCX_PIN_HEAD(lm_[sl]);
      MPCX_PIN_HEAD(gv_[sl]); MPCX_PIN_HEAD(sv_[sl]); MPCX_PIN_HEAD(vl_[sl]); MPCX_PIN_HEAD(vu_[sl]);
    }
#pragma unroll
    for (int sl = 0; sl < VS; ++sl) {
      const unsigned vb = vcls_slot(vw, sl);
      const double lo = lo_[sl], hi = hi_[sl], xv = xv_[sl], zl = zl_[sl], zu = zu_[sl];
      const double gr = gr_[sl], jt = jt_[sl];
      // on: NX <= i < NW and lo != hi; a fixed variable (lo == hi: every x_0 entry) has no barrier
      // terms (its psx is stored as 0)
      const bool on = (vb & VFREE) != 0u;
      const double rl = rcp_or0(on && (vb & VLO), xv - lo), ru = rcp_or0(on && (vb & VHI), hi - xv);
      pr0[sl] = on ? -(obj_scale * gr + jt) : 0.0;
      pr1[sl] = on ? rl - ru : 0.0;
      psx[sl] = on ? zl * rl + zu * ru : 0.0;  // sigma_x_v
      if (on) {
        const double rd = obj_scale * gr + jt - zl + zu;
        dmax = fmax(dmax, fabs(rd));
        dmax_u = fmax(dmax_u, fabs(rd) / obj_scale);
        if (vb & VLO) { const double pr = (xv - lo) * zl; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); zsum += fabs(zl); nz++; }
        if (vb & VHI) { const double pr = (hi - xv) * zu; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); zsum += fabs(zu); nz++; }
      }
    }
#pragma unroll
    for (int sl = 0; sl < CS; ++sl) {
      const int c = lane + sl * WAVE;
      const double lbv = lb_[sl], slo = sl_[sl], sup = su_[sl], gsc = gs_[sl], lm = lm_[sl];
      const double gvv = gv_[sl], sv = sv_[sl], vl = vl_[sl], vu = vu_[sl];
      const int cl = cls_slot(cw, sl);
      {
        const double rsl = rcp_or0(cl == 1 && isfin(slo), sv - slo), rsu = rcp_or0(cl == 1 && isfin(sup), sup - sv);
        const double sg = vl * rsl + vu * rsu;  // sigma_s_v
        const double rsg = rcp_or0(cl == 1, sg);
        const double r = (cl == 0) ? -(gvv - gsc * lbv) : -(gvv - sv);
        dq0[sl] = (cl == 1) ? r + lm * rsg : r;
        dq1[sl] = (cl == 1) ? (rsu - rsl) * rsg : 0.0;
        ddg[sl] = (cl == 0) ? -0.0 : (cl == 2) ? -1.0 : -rsg;  // -dual_diag_v at delta_w = delta_c = 0
      }
      if (c < M) {
        double cv, vv = 0.0;
        if (cl == 0) {
          cv = gvv - gsc * lbv;
          vv = fabs(cv);
        } else {
          cv = gvv - sv;
          if (cl == 1) {
            const double rs = -lm - vl + vu;
            dmax = fmax(dmax, fabs(rs));
            dmax_u = fmax(dmax_u, fabs(rs) * gsc / obj_scale);
            vv = fmax(0.0, fmax(slo - gvv, gvv - sup));
            if (isfin(slo)) { const double pr = (sv - slo) * vl; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); zsum += fabs(vl); nz++; }
            if (isfin(sup)) { const double pr = (sup - sv) * vu; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); zsum += fabs(vu); nz++; }
          }
        }
        pmax = fmax(pmax, fabs(cv));
        vmax_u = fmax(vmax_u, vv / gsc);
        lsum += fabs(lm);
      }
    }
    SPROF(6);  // loads and the per-element terms
    OptErr e;
    e.dual = wmax(dmax); e.dual_u = wmax(dmax_u); e.primal = wmax(pmax); e.viol_u = wmax(vmax_u);
    e.pmx = wmax(pmx); e.pmn = wmin(pmn);
    lsum = wsum(lsum); zsum = wsum(zsum); nz = wsumi(nz);
    e.ncompl = nz;
    const double smax = 100.0;
    // IPOPT: s_d over all multipliers (y_c, y_d, z_L, z_U, v_L, v_U)
    e.s_d = fmax(smax, (lsum + zsum) / fmax(1.0, (double)(M + nz))) / smax;
    e.s_c = nz > 0 ? fmax(smax, zsum / (double)nz) / smax : 1.0;
    K.e0 = e;
    SPROF(7);  // reductions
  }
  // ---- termination tests ----
  {
    const OptErr e0 = K.e0;
    const double fx = K.fx;
    const double err0 = e0.err_at(0.0);
    if (!(err0 == err0) || !(fx == fx)) { K.status = MPCX_INVALID_NUMBER; return 1; }
    // IPOPT OptimalityErrorConvergenceCheck::CheckConvergence (square problems: the dual
    // infeasibility and complementarity tolerances are lifted)
    if (err0 <= ka.opt.tol && e0.viol_u <= ka.opt.constr_viol_tol &&
        (K.square || (e0.dual_u <= ka.opt.dual_inf_tol && e0.compl_at(0.0) / obj_scale <= ka.opt.compl_inf_tol))) {
      K.status = MPCX_SOLVE_SUCCEEDED;
      return 1;
    }
    Acceptable acc = K.acc;
    if (ka.opt.acceptable_iter > 0 && current_is_acceptable(acc, e0, err0, fx, K.it, obj_scale, K.square, ka.opt)) {
      acc.count++;
      K.acc = acc;
      if (acc.count >= ka.opt.acceptable_iter) { K.status = MPCX_SOLVED_TO_ACCEPTABLE; return 1; }
    } else {
      acc.count = 0;
      K.acc = acc;
    }
    if (K.it >= ka.opt.max_iter) return 1;
  }
  // ---- barrier parameter update (monotone Fiacco-McCormick) ----
#pragma unroll 1
  for (int mu_up = 0; mu_up < 64; ++mu_up) {
    const double mu = K.mu;
    if (K.e0.err_at(mu) > ka.opt.kappa_eps * mu || mu <= ka.opt.mu_min) break;
    // IPOPT MonotoneMuUpdate::CalcNewMuAndTau: floor min(tol, compl_inf_tol) / (barrier_tol_factor + 1)
    const double new_mu = fmax(fmax(fmin(ka.opt.tol, ka.opt.compl_inf_tol) / (ka.opt.kappa_eps + 1.0), ka.opt.mu_min),
                               fmin(ka.opt.kappa_mu * mu, ka.opt.theta_mu == 1.5 ? mu * sqrt(mu) : pow_ool(mu, ka.opt.theta_mu)));
    if (new_mu == mu) break;  // IPOPT MonotoneMuUpdate: done when mu no longer changes
    K.mu = new_mu;
    K.tau = fmax(ka.opt.tau_min, 1.0 - new_mu);
    K.nfilt = 0;
    K.nsp[0] = 0;  // the filter is reset with mu (both parts)
  }
  SPROF(8);  // termination tests, barrier update
  const double mu = K.mu;
  // ---- Newton rhs and diagonal terms (rhs_dual with delta_w = delta_c = 0) ----
#pragma unroll
  for (int sl = 0; sl < VS; ++sl) {
    const int i = lane + sl * WAVE;
    if (i >= NX && i < NW) {
      const double r = pr0[sl] + mu * pr1[sl];
      const int b = (i - NX) / NP, off = (i - NX) % NP;
      const int li = off < NV ? off : LX1 + off - NV;
      a.rhs(b)[off] = r;
      a.dg(b)[li] = psx[sl];
    }
  }
#pragma unroll
  for (int sl = 0; sl < CS; ++sl) {
    const int c = lane + sl * WAVE;
    if (c < M) {
      const double rr = dq0[sl] - mu * dq1[sl];
      a.rhs(c / NG)[NP + c % NG] = rr;
      a.dg(c / NG)[crow(c % NG)] = ddg[sl];
    }
  }
  sync();
  SPROF(9);  // rhs / diagonal stores and the barrier
  return 0;
}


// ===========================================================================
// Soft restoration step and feasibility restoration phase (IPOPT's answer to a failed
// filter line search; oracle/ipm.py restates both step for step).
//
// Soft restoration (BacktrackingLineSearch::TrySoftRestoStep): the full fraction-to-the-
// boundary step with one step size for primal and dual variables, accepted if the original
// filter criterion holds at alpha = 0 or the primal-dual system error drops by 0.9999;
// a step accepted only by the error test keeps the solver in the soft phase (at most 10
// iterations), whose steps are tried the same way without backtracking.
//
// Restoration phase (MinC_1NrmRestorationPhase): a second interior-point run on
//   min rho sum(p + n) + zeta(mu)/2 ||D_R (x - x_R)||^2  s.t.  c~(x) - p + n = c~_L / in [d~_L, d~_U]
// (rho = 1000, zeta = sqrt(mu), D_R = diag(1 / max(1, |x_R|))), with p, n >= 0 eliminated
// from every KKT system: the stage factorisation sees the same structure, each constraint
// row's dual diagonal grows by 1/(Sigma_p + dw) + 1/(Sigma_n + dw) and its rhs by the p / n
// residuals.  It returns to the original problem once the original constraint violation has
// dropped by 0.9 and the point is acceptable to the original filter (RestoConvergenceCheck);
// bound multipliers then take one Newton step for complementarity over the whole primal
// change (reset to 1 above 1000), constraint multipliers restart at zero.  A restoration
// that converges on its own terms is a point of local infeasibility.
// ===========================================================================

// stationarity residuals of the restoration variables p, n: r_p = rho - lambda - mu/p and
// r_n = rho + lambda - mu/n.  Where p (n) is large, z = mu/p is small and lambda ~ -+rho, so the
// sum rho -+ lambda cancels; divided by Sigma_p = z/p ~ mu/p^2 its rounding error (eps rho)
// grows like p^2/mu and the eliminated p, n steps stop satisfying the linearised constraints
// (the restoration's own infeasibility then grows as mu falls).  The sum is formed exactly
// (two-sum), so the error is eps times the small residual itself.
__device__ __forceinline__ double resto_r(double lam_signed, double mu_over) {
  const double s = RESTO_RHO + lam_signed;
  const double bv = s - RESTO_RHO;
  const double err = (RESTO_RHO - (s - bv)) + (lam_signed - bv);
  return (s - mu_over) + err;
}

__device__ __forceinline__ double dr2_of(double xr) {
  const double d = 1.0 / fmax(1.0, fabs(xr));
  return d * d;
}

// IPOPT primal_dual_system_error at the current point (1-norms of the dual infeasibility,
// the constraint violation and the mu-complementarity; the common normalisation cancels in
// the soft-restoration ratio), from that point's derivative arrays
__device__ __noinline__ double pd_error(const Agent a, double mu, double obj_scale) {
  const int lane = lane_now();
  double e = 0.0;
  for (int i = NX + lane; i < NW; i += WAVE) {
    const double lo = a.xL()[i], hi = a.xU()[i];
    if (lo == hi) continue;
    const double xv = a.x()[i], zl = a.zL()[i], zu = a.zU()[i];
    e += fabs(obj_scale * acc_grad(a, i) + acc_jtl(a, i) - zl + zu);
    if (isfin(lo)) e += fabs((xv - lo) * zl - mu);
    if (isfin(hi)) e += fabs((hi - xv) * zu - mu);
  }
  for (int c = lane; c < M; c += WAVE) {
    const double lbv = a.lb()[c], ubv = a.ub()[c], slo = a.sL()[c], sup = a.sU()[c];
    const int cl = cls_of(lbv, ubv, slo, sup);
    const double gvv = a.gv()[c], sv = a.s()[c];
    e += fabs(cl == 0 ? gvv - a.gs()[c] * lbv : gvv - sv);
    if (cl == 1) {
      const double vl = a.vL()[c], vu = a.vU()[c];
      e += fabs(-a.lam()[c] - vl + vu);
      if (isfin(slo)) e += fabs((sv - slo) * vl - mu);
      if (isfin(sup)) e += fabs((sup - sv) * vu - mu);
    }
  }
  return wsum(e);
}

// iterate <-> backup (x, s, lambda, z, v, scaled g): the soft step's tentative trial
__device__ __noinline__ void iterate_copy(const Agent a, int to_backup) {
  const int lane = lane_now();
  for (int i = lane; i < NW; i += WAVE) {
    if (to_backup) { a.xr()[i] = a.x()[i]; a.zl0()[i] = a.zL()[i]; a.zu0()[i] = a.zU()[i]; }
    else { a.x()[i] = a.xr()[i]; a.zL()[i] = a.zl0()[i]; a.zU()[i] = a.zu0()[i]; }
  }
  for (int c = lane; c < M; c += WAVE) {
    if (to_backup) {
      a.sr()[c] = a.s()[c]; a.lr()[c] = a.lam()[c]; a.gvr()[c] = a.gv()[c];
      a.vl0()[c] = a.vL()[c]; a.vu0()[c] = a.vU()[c];
    } else {
      a.s()[c] = a.sr()[c]; a.lam()[c] = a.lr()[c]; a.gv()[c] = a.gvr()[c];
      a.vL()[c] = a.vl0()[c]; a.vU()[c] = a.vu0()[c];
    }
  }
  sync();
}

// the soft trial (xt, gt in LDS) with the same step size alpha for every variable,
// bound multipliers NOT yet corrected (IPOPT corrects them after acceptance)
__device__ __noinline__ void soft_apply(const Agent a, double mu, double alpha) {
  const int lane = lane_now();
  for (int i = NX + lane; i < NW; i += WAVE) {
    const double lo = a.xL()[i], hi = a.xU()[i];
    if (lo == hi) continue;
    const double xold = a.x()[i], d = a.dx()[i];
    a.x()[i] = gL.u.t.xt[i];
    if (isfin(lo)) { const double zl = a.zL()[i], sl0 = xold - lo; a.zL()[i] = zl + alpha * (mu / sl0 - zl - (zl / sl0) * d); }
    if (isfin(hi)) { const double zu = a.zU()[i], su0 = hi - xold; a.zU()[i] = zu + alpha * (mu / su0 - zu + (zu / su0) * d); }
  }
  for (int c = lane; c < M; c += WAVE) {
    const double lbv = a.lb()[c], ubv = a.ub()[c], slo = a.sL()[c], sup = a.sU()[c];
    const double sold = a.s()[c], dsv = a.ds()[c];
    a.lam()[c] += alpha * a.dl()[c];
    a.gv()[c] = gL.u.t.gt[c];
    a.s()[c] = sold + alpha * dsv;
    if (cls_of(lbv, ubv, slo, sup) != 1) continue;
    if (isfin(slo)) { const double vl = a.vL()[c], s0 = sold - slo; a.vL()[c] = vl + alpha * (mu / s0 - vl - (vl / s0) * dsv); }
    if (isfin(sup)) { const double vu = a.vU()[c], s0 = sup - sold; a.vU()[c] = vu + alpha * (mu / s0 - vu + (vu / s0) * dsv); }
  }
  sync();
}

// kappa_sigma correction of the bound multipliers at the current point
__device__ __noinline__ void sigma_clip(const Agent a, double kappa_sigma, double mu) {
  const int lane = lane_now();
  for (int i = NX + lane; i < NW; i += WAVE) {
    const double lo = a.xL()[i], hi = a.xU()[i], xv = a.x()[i];
    if (lo == hi) continue;
    if (isfin(lo)) { const double s_l = xv - lo; a.zL()[i] = fmax(fmin(a.zL()[i], kappa_sigma * mu / s_l), mu / (kappa_sigma * s_l)); }
    if (isfin(hi)) { const double s_u = hi - xv; a.zU()[i] = fmax(fmin(a.zU()[i], kappa_sigma * mu / s_u), mu / (kappa_sigma * s_u)); }
  }
  for (int c = lane; c < M; c += WAVE) {
    const double slo = a.sL()[c], sup = a.sU()[c], sv = a.s()[c];
    if (cls_of(a.lb()[c], a.ub()[c], slo, sup) != 1) continue;
    if (isfin(slo)) { const double s_l = sv - slo; a.vL()[c] = fmax(fmin(a.vL()[c], kappa_sigma * mu / s_l), mu / (kappa_sigma * s_l)); }
    if (isfin(sup)) { const double s_u = sup - sv; a.vU()[c] = fmax(fmin(a.vU()[c], kappa_sigma * mu / s_u), mu / (kappa_sigma * s_u)); }
  }
  sync();
}

// TrySoftRestoStep.  0: rejected (iterate unchanged); 1: accepted by the original filter
// criterion (the caller takes the trial as a regular step); 2: accepted by the
// primal-dual error test (trial applied, multipliers corrected, derivatives evaluated)
__device__ __noinline__ int soft_try(const Agent a) {
  KArgs* const argp = kargs();
  KState& K = gL.ks;
  K.lsmode = 1;
  line_search(a);
  K.lsmode = 0;
  K.n_trials += K.ls.trials;
  if (K.ls.accepted) return 1;
  const Trial tr = K.ls.tr;
  if (!(isfin(tr.theta) && isfin(tr.phi))) return 0;
  const double pd0 = pd_error(a, K.mu, K.obj_scale);
  iterate_copy(a, 1);
  soft_apply(a, K.mu, K.ls.alpha);
  eval_gj_lds(a);
  sync();
  const double pd1 = pd_error(a, K.mu, K.obj_scale);
  if (pd1 <= SOFT_PD_FACTOR * pd0) {
    sigma_clip(a, (*argp).opt.kappa_sigma, K.mu);
    return 2;
  }
  iterate_copy(a, 0);
  eval_gj_ws(a, a.x(), gL.want_sdh);
  sync();
  return 0;
}

// The current filter's spill list (tier = K.resto): its entries older than the MAXF in LDS.
__device__ __forceinline__ cdbl* fsp_tier(int tier) { return cold_base() + O_FSP + 2L * FSPILL * tier; }

// a trial (th, ph) dominated by an entry of the current filter's spill list (wave-uniform)
__device__ __noinline__ bool spill_dominates(double th, double ph) {
  KState& K = gL.ks;
  const int t = K.resto, ns = K.nsp[t];
  cdbl* sp = fsp_tier(t);
  const int lane = lane_now();
  bool dom = false;
  for (int b = 0; b < ns; b += WAVE) {
    const int j = b + lane;
    if (j < ns && th >= sp[j] && ph >= sp[FSPILL + j]) dom = true;
  }
  return __any(dom);
}

// remove the spill entries (th, ph) dominates, order kept; returns the new count.  Each lane
// writes at or below the index it read, after the whole chunk was read.
__device__ __noinline__ int spill_prune(double th, double ph, int t, int ns) {
  cdbl* sp = fsp_tier(t);
  const int lane = lane_now();
  int out = 0;
  for (int b = 0; b < ns; b += WAVE) {
    const int j = b + lane;
    double e = 0.0, p = 0.0;
    if (j < ns) { e = sp[j]; p = sp[FSPILL + j]; }
    const bool keep = j < ns && !(th <= e && ph <= p);
    const unsigned long long km = __ballot(keep);
    const int pos = out + __popcll(km & ((1ull << lane) - 1ull));
    wsync();
    if (keep) { sp[pos] = e; sp[FSPILL + pos] = p; }
    wsync();
    out += __popcll(km);
  }
  return out;
}

// drop the oldest spill entry (a full filter), order kept
__device__ __noinline__ void spill_shift(int t, int ns) {
  cdbl* sp = fsp_tier(t);
  const int lane = lane_now();
  for (int b = 1; b < ns; b += WAVE) {
    const int j = b + lane;
    double e = 0.0, p = 0.0;
    if (j < ns) { e = sp[j]; p = sp[FSPILL + j]; }
    wsync();
    if (j < ns) { sp[j - 1] = e; sp[FSPILL + j - 1] = p; }
    wsync();
  }
}

// IPOPT Filter::AddEntry of (th, ph): the entries the new one dominates (th <= theta_j and
// ph <= phi_j) are removed from both parts, order kept, then it is appended to the LDS part; when
// the LDS part is still full its oldest entry moves to the end of the spill list, and a full spill
// list first drops its own oldest entry (counted: IPOPT's list is unbounded).  One LDS entry per
// lane: a ballot compacts the kept entries in one LDS read and write.
__device__ __forceinline__ void filter_insert(double th, double ph) {
  KState& K = gL.ks;
  const int j = lane_now();
  const int t = K.resto;
  int ns = K.nsp[t];
  if (ns > 0) ns = spill_prune(th, ph, t, ns);
  const int nf = K.nfilt;
  const double ej = gL.fth[j < MAXF ? j : 0], pj = gL.fph[j < MAXF ? j : 0];
  const bool keep = j < nf && !(th <= ej && ph <= pj);
  const unsigned long long km = __ballot(keep);
  int nk = __popcll(km);
  int pos = __popcll(km & ((1ull << j) - 1ull));
  const int full = nk >= MAXF ? 1 : 0;  // the oldest kept entry leaves the LDS part
  if (full) {
    const int first = __builtin_ctzll(km);
    const double e0 = rl_f64(ej, first), p0 = rl_f64(pj, first);
    if (FSPILL == 0) {
      K.n_filt_over += 1;
    } else {
      if (ns >= FSPILL) { spill_shift(t, ns); ns -= 1; K.n_filt_over += 1; }
      cdbl* sp = fsp_tier(t);
      if (j == 0) { sp[ns] = e0; sp[FSPILL + ns] = p0; }
      ns += 1;
    }
  }
  pos -= full;
  nk -= full;
  wsync();
  if (keep && pos >= 0) { gL.fth[pos] = ej; gL.fph[pos] = pj; }
  if (j == 0) { gL.fth[nk] = th; gL.fph[nk] = ph; }
  wsync();
  K.nfilt = nk + 1;
  K.nsp[t] = ns;
}

// ---- restoration phase ----------------------------------------------------------------

// start: called at the iterate whose line search (and soft step) failed, with K.st of it
__device__ __noinline__ void resto_start(const Agent a) {
  KArgs* const argp = kargs();
  KArgs& ka = *argp;
  KState& K = gL.ks;
  const int lane = lane_now();
  {  // FilterLSAcceptor::PrepareRestoPhaseStart: the current point enters the original filter
    const double theta = K.st.theta, phi = K.fx - K.mu * K.st.barrier;
    filter_insert((1.0 - ka.opt.gamma_theta) * theta, phi - ka.opt.gamma_phi * theta);
    const int nfilt = K.nfilt;
    for (int j = lane; j < nfilt; j += WAVE) { a.flt0()[j] = gL.fth[j]; a.flt0()[MAXF + j] = gL.fph[j]; }
    K.nfilt0 = nfilt;
    K.theta_start = theta;
  }
  K.theta_max0 = K.theta_max; K.theta_min0 = K.theta_min;
  K.mu0 = K.mu; K.tau0 = K.tau; K.dw_last0 = K.dw_last; K.acc0 = K.acc;
  K.fo = K.fx;
  double cmax = 0.0;
  for (int c = lane; c < M; c += WAVE) {
    const int cl = cls_of(a.lb()[c], a.ub()[c], a.sL()[c], a.sU()[c]);
    cmax = fmax(cmax, fabs(cl == 0 ? a.gv()[c] - a.gs()[c] * a.lb()[c] : a.gv()[c] - a.s()[c]));
  }
  const double mu_r = fmax(K.mu, wmax(cmax));
  double pn = 0.0, th = 0.0;
  int nfree = 0, neq = 0;
  for (int i = lane; i < NW; i += WAVE) {
    a.xr()[i] = a.x()[i];
    const double zl = a.zL()[i], zu = a.zU()[i];
    a.zl0()[i] = zl; a.zu0()[i] = zu;
    a.zL()[i] = fmin(zl, RESTO_RHO);
    a.zU()[i] = fmin(zu, RESTO_RHO);
    nfree += (i >= NX && a.xL()[i] != a.xU()[i]) ? 1 : 0;
  }
  for (int c = lane; c < M; c += WAVE) {
    const int cl = cls_of(a.lb()[c], a.ub()[c], a.sL()[c], a.sU()[c]);
    const double cv = cl == 0 ? a.gv()[c] - a.gs()[c] * a.lb()[c] : a.gv()[c] - a.s()[c];
    // p, n solving the restoration problem's complementarity at its start (W&B 2006, eq. 33)
    const double q = (mu_r - RESTO_RHO * cv) / (2.0 * RESTO_RHO);
    const double nv = q + sqrt(q * q + mu_r * cv / (2.0 * RESTO_RHO));
    const double pv = cv + nv;
    a.rp()[c] = pv; a.rn()[c] = nv;
    a.rzp()[c] = mu_r / pv; a.rzn()[c] = mu_r / nv;
    pn += pv + nv;
    th += fabs(cv - pv + nv);
    a.sr()[c] = a.s()[c];
    const double vl = a.vL()[c], vu = a.vU()[c];
    a.vl0()[c] = vl; a.vu0()[c] = vu;
    a.vL()[c] = fmin(vl, RESTO_RHO);
    a.vU()[c] = fmin(vu, RESTO_RHO);
    a.lam()[c] = 0.0;
    neq += cl == 0 ? 1 : 0;
  }
  pn = wsum(pn);
  th = wsum(th);
#ifdef MPCX_TRACE_IT  // diagnostics: the smallest slacks at the restoration start
  {
    double mxl = INFINITY, mxu = INFINITY, msl = INFINITY, msu = INFINITY, mp = INFINITY, mn = INFINITY;
    for (int i = NX + lane; i < NW; i += WAVE) {
      const double lo = a.xL()[i], hi = a.xU()[i], xv = a.x()[i];
      if (lo == hi) continue;
      if (isfin(lo)) mxl = fmin(mxl, xv - lo);
      if (isfin(hi)) mxu = fmin(mxu, hi - xv);
    }
    for (int c = lane; c < M; c += WAVE) {
      const double slo = a.sL()[c], sup = a.sU()[c], sv = a.s()[c];
      if (cls_of(a.lb()[c], a.ub()[c], slo, sup) == 1) {
        if (isfin(slo)) msl = fmin(msl, sv - slo);
        if (isfin(sup)) msu = fmin(msu, sup - sv);
      }
      mp = fmin(mp, a.rp()[c]); mn = fmin(mn, a.rn()[c]);
    }
    mxl = wmin(mxl); mxu = wmin(mxu); msl = wmin(msl); msu = wmin(msu); mp = wmin(mp); mn = wmin(mn);
    if (lane == 0)
      printf("mpcx resto-start it=%d mu_r=%.6e pn=%.6e th=%.6e min x-lo=%.3e hi-x=%.3e s-sL=%.3e sU-s=%.3e p=%.3e n=%.3e\n",
             K.it, mu_r, pn, th, mxl, mxu, msl, msu, mp, mn);
  }
#endif
  K.square_r = (wsumi(nfree) + 2 * M) == wsumi(neq);
  sync();
  eval_gj_ws(a, a.x(), gL.want_sdh);  // (J~^T lambda) with lambda = 0
  sync();
  K.mu = mu_r;
  K.tau = fmax(ka.opt.tau_min, 1.0 - mu_r);
  K.zeta = sqrt(mu_r);
  K.fx = RESTO_RHO * pn;  // x = x_R: no proximity term yet
  K.theta_max = ka.opt.theta_max_fact * fmax(1.0, th);
  K.theta_min = ka.opt.theta_min_fact * fmax(1.0, th);
  K.nfilt = 0;
  K.nsp[1] = 0;  // the restoration phase's own filter; the problem's (LDS part saved, spill kept) returns with it
  K.dw_last = 0.0;
  K.acc = Acceptable{-1e50, -1e50, -1, 0};
  K.resto = 1;
  K.soft = 0;
  K.soft_count = 0;
  K.n_fallback += 1;
}

// back to the original problem (the restoration iterate passed the return test)
__device__ __noinline__ void resto_return(const Agent a) {
  KArgs* const argp = kargs();
  KState& K = gL.ks;
  const int lane = lane_now();
  const double mu0 = K.mu0, tau0 = K.tau0;
  // one Newton step for complementarity over the whole primal change, fraction to the boundary
  double ad = 1.0;
  for (int i = NX + lane; i < NW; i += WAVE) {
    const double lo = a.xL()[i], hi = a.xU()[i];
    if (lo == hi) continue;
    const double xv = a.x()[i], x0 = a.xr()[i];
    if (isfin(lo)) { const double z0 = a.zl0()[i], dz = (mu0 - z0 * (xv - lo)) / (x0 - lo); if (dz < 0) ad = fmin(ad, -tau0 * z0 / dz); }
    if (isfin(hi)) { const double z0 = a.zu0()[i], dz = (mu0 - z0 * (hi - xv)) / (hi - x0); if (dz < 0) ad = fmin(ad, -tau0 * z0 / dz); }
  }
  for (int c = lane; c < M; c += WAVE) {
    const double slo = a.sL()[c], sup = a.sU()[c];
    if (cls_of(a.lb()[c], a.ub()[c], slo, sup) != 1) continue;
    const double sv = a.s()[c], s0 = a.sr()[c];
    if (isfin(slo)) { const double v0 = a.vl0()[c], dv = (mu0 - v0 * (sv - slo)) / (s0 - slo); if (dv < 0) ad = fmin(ad, -tau0 * v0 / dv); }
    if (isfin(sup)) { const double v0 = a.vu0()[c], dv = (mu0 - v0 * (sup - sv)) / (sup - s0); if (dv < 0) ad = fmin(ad, -tau0 * v0 / dv); }
  }
  ad = wmin(ad);
  double zmax = 0.0;
  for (int i = NX + lane; i < NW; i += WAVE) {
    const double lo = a.xL()[i], hi = a.xU()[i];
    if (lo == hi) continue;
    const double xv = a.x()[i], x0 = a.xr()[i];
    if (isfin(lo)) { const double z0 = a.zl0()[i], z = z0 + ad * (mu0 - z0 * (xv - lo)) / (x0 - lo); a.zL()[i] = z; zmax = fmax(zmax, fabs(z)); }
    if (isfin(hi)) { const double z0 = a.zu0()[i], z = z0 + ad * (mu0 - z0 * (hi - xv)) / (hi - x0); a.zU()[i] = z; zmax = fmax(zmax, fabs(z)); }
  }
  for (int c = lane; c < M; c += WAVE) {
    const double slo = a.sL()[c], sup = a.sU()[c];
    a.lam()[c] = 0.0;  // constr_mult_reset_threshold = 0: constraint multipliers restart at zero
    if (cls_of(a.lb()[c], a.ub()[c], slo, sup) != 1) continue;
    const double sv = a.s()[c], s0 = a.sr()[c];
    if (isfin(slo)) { const double v0 = a.vl0()[c], v = v0 + ad * (mu0 - v0 * (sv - slo)) / (s0 - slo); a.vL()[c] = v; zmax = fmax(zmax, fabs(v)); }
    if (isfin(sup)) { const double v0 = a.vu0()[c], v = v0 + ad * (mu0 - v0 * (sup - sv)) / (sup - s0); a.vU()[c] = v; zmax = fmax(zmax, fabs(v)); }
  }
  zmax = wmax(zmax);
  if (zmax > BOUND_MULT_RESET) {
    for (int i = NX + lane; i < NW; i += WAVE) {
      const double lo = a.xL()[i], hi = a.xU()[i];
      if (lo == hi) continue;
      a.zL()[i] = isfin(lo) ? 1.0 : 0.0;
      a.zU()[i] = isfin(hi) ? 1.0 : 0.0;
    }
    for (int c = lane; c < M; c += WAVE) {
      const double slo = a.sL()[c], sup = a.sU()[c];
      if (cls_of(a.lb()[c], a.ub()[c], slo, sup) != 1) continue;
      a.vL()[c] = isfin(slo) ? 1.0 : 0.0;
      a.vU()[c] = isfin(sup) ? 1.0 : 0.0;
    }
  }
  const int nfilt = K.nfilt0;
  for (int j = lane; j < nfilt; j += WAVE) { gL.fth[j] = a.flt0()[j]; gL.fph[j] = a.flt0()[MAXF + j]; }
  sync();
  eval_gj_ws(a, a.x(), gL.want_sdh);  // (J~^T lambda) with lambda = 0
  sync();
  K.nfilt = nfilt;
  K.mu = mu0; K.tau = tau0; K.dw_last = K.dw_last0; K.acc = K.acc0;
  K.theta_max = K.theta_max0; K.theta_min = K.theta_min0;
  K.fx = K.fo;
  K.resto = 0;
  K.soft = 0;
  K.soft_count = 0;
}

// Top of a restoration iteration: the return test, then the restoration problem's
// optimality error, termination tests, barrier update (zeta follows mu), Newton rhs and
// diagonal terms.  Returns 0 (rhs written), 1 (stop, K.status set), 2 (return test passed)
__device__ __noinline__ void rhs_dual_resto(const Agent a, double mu, double dw, double dc);
__device__ __noinline__ int iter_head_resto(const Agent a) {
  KArgs* const argp = kargs();
  KArgs& ka = *argp;
  KState& K = gL.ks;
  const int lane = lane_now();
  // primal rows: r = -(jt + zeta gdr) + mu pr1, diagonal psx + zeta dr2; dual residual of
  // x: zeta gdr + hj (zeta-dependent, kept per slot for the barrier loop)
  double gdr[VS], hj[VS], jtv[VS], pr1[VS], psx[VS], d2[VS];
  double dmax_r = 0.0, pmax = 0.0, vmax = 0.0, pmx = -INFINITY, pmn = INFINITY, lsum = 0.0, zsum = 0.0;
  double barx0 = 0.0, bars0 = 0.0, tho = 0.0, spn = 0.0, sd = 0.0;
  int nz = 0;
#pragma unroll
  for (int sl = 0; sl < VS; ++sl) {
    const int i = lane + sl * WAVE;
    const int ii = (i >= NX && i < NW) ? i : NX;
    const double lo = a.xL()[ii], hi = a.xU()[ii], xv = a.x()[ii], zl = a.zL()[ii], zu = a.zU()[ii];
    const double xrv = a.xr()[ii], jt = acc_jtl(a, ii);
    const bool on = i >= NX && i < NW && lo != hi;
    const double dr2 = dr2_of(xrv);
    gdr[sl] = on ? dr2 * (xv - xrv) : 0.0;
    hj[sl] = on ? jt - zl + zu : 0.0;
    jtv[sl] = jt;
    d2[sl] = on ? dr2 : 0.0;
    pr1[sl] = on ? (isfin(lo) ? 1.0 / (xv - lo) : 0.0) - (isfin(hi) ? 1.0 / (hi - xv) : 0.0) : 0.0;
    psx[sl] = sigma_x_v(xv, lo, hi, zl, zu);
    if (on) {
      sd += dr2 * (xv - xrv) * (xv - xrv);
      if (isfin(lo)) { const double pr = (xv - lo) * zl; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); zsum += fabs(zl); nz++; barx0 += log(xv - lo); }
      if (isfin(hi)) { const double pr = (hi - xv) * zu; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); zsum += fabs(zu); nz++; barx0 += log(hi - xv); }
    }
  }
#pragma unroll
  for (int sl = 0; sl < CS; ++sl) {
    const int c = lane + sl * WAVE;
    const int cc = c < M ? c : 0;
    const double lbv = a.lb()[cc], ubv = a.ub()[cc], slo = a.sL()[cc], sup = a.sU()[cc];
    const double gsc = a.gs()[cc], gvv = a.gv()[cc], sv = a.s()[cc], lm = a.lam()[cc];
    const double vl = a.vL()[cc], vu = a.vU()[cc];
    const double pv = a.rp()[cc], nv = a.rn()[cc], zp = a.rzp()[cc], zn = a.rzn()[cc];
    const int cl = cls_of(lbv, ubv, slo, sup);
    const double co = (cl == 0) ? gvv - gsc * lbv : gvv - sv;   // original residual
    const double cr = co - pv + nv;                               // restoration residual
    const double sg = sigma_s_v(sv, slo, sup, vl, vu);
    const double sgp = zp / pv, sgn = zn / nv;
    if (c < M) {
      tho += fabs(co);
      pmax = fmax(pmax, fabs(cr));
      dmax_r = fmax(dmax_r, fmax(fabs(RESTO_RHO - lm - zp), fabs(RESTO_RHO + lm - zn)));
      { const double pr = pv * zp; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); }
      { const double pr = nv * zn; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); }
      zsum += fabs(zp) + fabs(zn);
      nz += 2;
      spn += pv + nv;
      const double gr = gvv - pv + nv;
      if (cl == 0) {
        vmax = fmax(vmax, fabs(cr));
      } else if (cl == 1) {
        dmax_r = fmax(dmax_r, fabs(-lm - vl + vu));
        vmax = fmax(vmax, fmax(0.0, fmax(slo - gr, gr - sup)));
        if (isfin(slo)) { const double pr = (sv - slo) * vl; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); zsum += fabs(vl); nz++; bars0 += log(sv - slo); }
        if (isfin(sup)) { const double pr = (sup - sv) * vu; pmx = fmax(pmx, pr); pmn = fmin(pmn, pr); zsum += fabs(vu); nz++; bars0 += log(sup - sv); }
      }
      lsum += fabs(lm);
    }
  }
  // ---- return test (RestoConvergenceCheck) ----
  tho = wsum(tho);
  {
    const double bar = wsum(barx0) + wsum(bars0);
    bool ret = tho <= RESTO_KAPPA * K.theta_start;
    if (ret) {
      const double phio = K.fo - K.mu0 * bar;
      ret = tho <= K.theta_max0;
      const int nf = K.nfilt0;
      for (int j = 0; j < nf && ret; ++j)
        if (tho >= a.flt0()[j] && phio >= a.flt0()[MAXF + j]) ret = false;
      const int ns0 = K.nsp[0];  // the original filter's older entries (its spill list, untouched)
      for (int j = 0; j < ns0 && ret; ++j)
        if (tho >= a.fsp(0)[j] && phio >= a.fsp(0)[FSPILL + j]) ret = false;
    }
    if (ret) return 2;
  }
  OptErr e;
  dmax_r = wmax(dmax_r);
  auto dual_x = [&](double zeta) {
    double m = 0.0;
#pragma unroll
    for (int sl = 0; sl < VS; ++sl) m = fmax(m, fabs(zeta * gdr[sl] + hj[sl]));
    return fmax(dmax_r, wmax(m));
  };
  e.dual = dual_x(K.zeta); e.dual_u = e.dual;
  e.primal = wmax(pmax); e.viol_u = wmax(vmax);
  e.pmx = wmax(pmx); e.pmn = wmin(pmn);
  lsum = wsum(lsum); zsum = wsum(zsum); nz = wsumi(nz);
  spn = wsum(spn); sd = wsum(sd);
  e.ncompl = nz;
  e.s_d = fmax(100.0, (lsum + zsum) / fmax(1.0, (double)(M + nz))) / 100.0;
  e.s_c = nz > 0 ? fmax(100.0, zsum / (double)nz) / 100.0 : 1.0;
  K.e0 = e;
  K.fx = RESTO_RHO * spn + 0.5 * K.zeta * sd;
  {
    const double err0 = e.err_at(0.0);
    if (!(err0 == err0) || !(K.fx == K.fx)) { K.status = MPCX_INVALID_NUMBER; return 1; }
    if (err0 <= ka.opt.tol && e.viol_u <= ka.opt.constr_viol_tol &&
        (K.square_r || (e.dual_u <= ka.opt.dual_inf_tol && e.compl_at(0.0) <= ka.opt.compl_inf_tol))) {
      K.status = MPCX_INFEASIBLE;
      return 1;
    }
    Acceptable acc = K.acc;
    if (ka.opt.acceptable_iter > 0 && current_is_acceptable(acc, e, err0, K.fx, K.it, 1.0, K.square_r, ka.opt)) {
      acc.count++;
      K.acc = acc;
      if (acc.count >= ka.opt.acceptable_iter) { K.status = MPCX_INFEASIBLE; return 1; }
    } else {
      acc.count = 0;
      K.acc = acc;
    }
    if (K.it >= ka.opt.max_iter) return 1;
  }
  // ---- barrier update; the proximity weight follows mu ----
#pragma unroll 1
  for (int mu_up = 0; mu_up < 64; ++mu_up) {
    const double mu = K.mu;
    if (e.err_at(mu) > ka.opt.kappa_eps * mu || mu <= ka.opt.mu_min) break;
    const double new_mu = fmax(fmax(fmin(ka.opt.tol, ka.opt.compl_inf_tol) / (ka.opt.kappa_eps + 1.0), ka.opt.mu_min),
                               fmin(ka.opt.kappa_mu * mu, ka.opt.theta_mu == 1.5 ? mu * sqrt(mu) : pow_ool(mu, ka.opt.theta_mu)));
    if (new_mu == mu) break;
    K.mu = new_mu;
    K.tau = fmax(ka.opt.tau_min, 1.0 - new_mu);
    K.nfilt = 0;
    K.nsp[1] = 0;
    K.zeta = sqrt(new_mu);
    K.fx = RESTO_RHO * spn + 0.5 * K.zeta * sd;
    e.dual = dual_x(K.zeta);
  }
  const double mu = K.mu, zeta = K.zeta;
#pragma unroll
  for (int sl = 0; sl < VS; ++sl) {
    const int i = lane + sl * WAVE;
    if (i >= NX && i < NW) {
      const bool on = a.xL()[i] != a.xU()[i];
      const double r = on ? -(jtv[sl] + zeta * gdr[sl]) + mu * pr1[sl] : 0.0;
      const int b = (i - NX) / NP, off = (i - NX) % NP;
      const int li = off < NV ? off : LX1 + off - NV;
      a.rhs(b)[off] = r;
      a.dg(b)[li] = psx[sl] + zeta * d2[sl];
    }
  }
  // dual rows at the final mu, in the same arithmetic as the inertia-correction pass and the
  // step recovery (the affine split dq0 - mu dq1 would round r_p / r_n differently)
  rhs_dual_resto(a, mu, 0.0, 0.0);
  return 0;
}

// dual rows of the restoration rhs with the inertia-correction terms (delta_w, delta_c)
__device__ __noinline__ void rhs_dual_resto(const Agent a, double mu, double dw, double dc) {
  const int lane = lane_now();
  for (int c = lane; c < M; c += WAVE) {
    const double lbv = a.lb()[c], ubv = a.ub()[c], slo = a.sL()[c], sup = a.sU()[c];
    const double gvv = a.gv()[c], gsc = a.gs()[c], sv = a.s()[c], lm = a.lam()[c];
    const double vl = a.vL()[c], vu = a.vU()[c];
    const double pv = a.rp()[c], nv = a.rn()[c], sgp = a.rzp()[c] / pv + dw, sgn = a.rzn()[c] / nv + dw;
    const int cl = cls_of(lbv, ubv, slo, sup);
    const double sg = sigma_s_v(sv, slo, sup, vl, vu);
    double rr = -((cl == 0 ? gvv - gsc * lbv : gvv - sv) - pv + nv);
    if (cl == 1) {
      double gphis = 0.0;
      if (isfin(slo)) gphis -= mu / (sv - slo);
      if (isfin(sup)) gphis += mu / (sup - sv);
      rr -= (gphis - lm) / (sg + dw);
    }
    rr += -resto_r(-lm, mu / pv) / sgp + resto_r(lm, mu / nv) / sgn;
    a.rhs(c / NG)[NP + c % NG] = rr;
    a.dg(c / NG)[crow(c % NG)] = -(dual_diag_v(cl, sg, KKTDiag{dw, dc, NEWTON}) + 1.0 / sgp + 1.0 / sgn);
  }
  sync();
}

// ---- iterative refinement of the restoration step (IPOPT PDFullSpaceSolver::Solve) -------
// The restoration KKT system is solved with p and n eliminated (their diagonal terms folded
// into the constraint rows, as IPOPT's AugRestoSystemSolver does); IPOPT then refines the
// step on the FULL system, p and n explicit.  Where a row stays violated Sigma_p = z_p / p is
// tiny and dp = (dlam - r_p) / (Sigma_p + dw) amplifies the rounding of dlam, so the
// eliminated step alone misses the linearised constraints by far more than the direct solve
// of the full system does (profiles/r03/s2/resto_trace_case4_*.txt).  resto_resid forms the
// residual of the full system at the current step (gL.u.sol; dp, dn recovered from dlam) from
// the compact stage images and the diagonal terms, writes it as the next right-hand side and
// returns IPOPT's residual ratio; the kernel body re-factors (same matrix) and adds the
// correction, at least MIN_REFINE times and until the ratio is <= RESID_RATIO_MAX.

// local step vector of stage k at local index i (the step in block order, LDS)
__device__ __forceinline__ double loc_step(int k, int i) {
  const int ki = lkind(i);
  if (ki == 0) return gL.u.sol[k * NB + i];
  if (kdual(ki)) return gL.u.sol[k * NB + NP + lrow(i)];
  if (ki == 3) return gL.u.sol[k * NB + NV + (i - LX1)];
  if (ki == 2) return k > 0 ? gL.u.sol[(k - 1) * NB + NV + (i - NI)] : 0.0;
  return 0.0;
}

__device__ __noinline__ double resto_resid(const Agent a, int first) {
  KState& K = gL.ks;
  const double mu = K.mu, dw = K.dw, dc = K.dc;
  const int lane = lane_now();
  cdbl* const RU = a.ru();
  cdbl* const RY = a.ry();
  cdbl* const RR = a.rrhs();
  if (first)
    for (int t = lane; t < N * NB; t += WAVE) RR[t] = a.rhs(t / NB)[t % NB];
  // stage-local products y_k = A_k u_k of the off-diagonal entries and the primal diagonal
  // (lane k, stage k); the dual diagonal is applied below with p, n explicit
  for (int k = lane; k < N; k += WAVE) {
    const unsigned long long fm = gL.fixm[k];
    for (int i = 0; i < NLOC; ++i) { RU[k * NLOC + i] = loc_step(k, i); RY[k * NLOC + i] = 0.0; }
    const wdbl* src = a.lp(k);
    const wdbl* dg = a.dg(k);
#pragma unroll 1
    for (int t = 0; t < NCPT; ++t) {
      if (t >= CB && t < CB + NLOC) continue;  // border (rhs) entries
      const int ij = kCIJ[t], i = ij & 255, j = ij >> 8;
      if (i >= NLOC || j >= NLOC || (((fm >> i) | (fm >> j)) & 1ull)) continue;
      double v = src[t * N];
      if (i == j) {
        const int ki = lkind(i);
        if (kdual(ki)) continue;
        if (ki == 0 || ki == 3) v += dg[i] + dw;
        RY[k * NLOC + i] += v * RU[k * NLOC + i];
      } else {
        RY[k * NLOC + i] += v * RU[k * NLOC + j];
        RY[k * NLOC + j] += v * RU[k * NLOC + i];
      }
    }
  }
  sync();
  double nres = 0.0, nsol = 0.0, nrhs = 0.0;
  for (int i = NX + lane; i < NW; i += WAVE) {
    const int b = (i - NX) / NP, off = (i - NX) % NP;
    double y;
    if (off < NV) {
      y = RY[b * NLOC + off];
    } else {
      const int c = off - NV;
      y = RY[b * NLOC + LX1 + c] + (b + 1 < N ? RY[(b + 1) * NLOC + NI + c] : 0.0);
    }
    const double r0 = RR[b * NB + off];
    const double res = (a.xL()[i] == a.xU()[i]) ? 0.0 : r0 - y;
    a.rhs(b)[off] = res;
    nres = fmax(nres, fabs(res));
    nrhs = fmax(nrhs, fabs(r0));
    nsol = fmax(nsol, fabs(gL.u.sol[b * NB + off]));
  }
  for (int c = lane; c < M; c += WAVE) {
    const int b = c / NG, r = c % NG;
    const double lbv = a.lb()[c], ubv = a.ub()[c], slo = a.sL()[c], sup = a.sU()[c];
    const double gvv = a.gv()[c], gsc = a.gs()[c], sv = a.s()[c], lm = a.lam()[c];
    const double pv = a.rp()[c], nv = a.rn()[c], sgp = a.rzp()[c] / pv + dw, sgn = a.rzn()[c] / nv + dw;
    const int cl = cls_of(lbv, ubv, slo, sup);
    const double sg = sigma_s_v(sv, slo, sup, a.vL()[c], a.vU()[c]);
    double rl = -((cl == 0 ? gvv - gsc * lbv : gvv - sv) - pv + nv);
    if (cl == 1) {
      double gphis = 0.0;
      if (isfin(slo)) gphis -= mu / (sv - slo);
      if (isfin(sup)) gphis += mu / (sup - sv);
      rl -= (gphis - lm) / (sg + dw);
    }
    const double rpv = resto_r(-lm, mu / pv), rnv = resto_r(lm, mu / nv);
    const double dl = gL.u.sol[b * NB + NP + r];
    const double dp = (dl - rpv) / sgp, dn = (-dl - rnv) / sgn;
    const double dd = dual_diag_v(cl, sg, KKTDiag{dw, dc, NEWTON});
    const double res = rl - (RY[b * NLOC + crow(r)] - dp + dn - dd * dl);
    a.rhs(b)[NP + r] = res;
    nres = fmax(nres, fabs(res));
    nrhs = fmax(nrhs, fmax(fabs(rl), fmax(fabs(rpv), fabs(rnv))));
    nsol = fmax(nsol, fmax(fabs(dl), fmax(fabs(dp), fabs(dn))));
  }
  nres = wmax(nres);
  nsol = wmax(nsol);
  if (first) K.rnrm = wmax(nrhs);
  const double nr = K.rnrm;
  sync();
  return (nr + nsol == 0.0) ? nres : nres / (fmin(nsol, 1e6 * nr) + nr);
}

// the step so far <-> the workspace (the factorisation reuses the step's LDS)
__device__ __noinline__ void resto_step_io(const Agent a, int add) {
  const int lane = lane_now();
  for (int t = lane; t < N * NB; t += WAVE) {
    if (add) gL.u.sol[t] += a.rsol()[t];
    else a.rsol()[t] = gL.u.sol[t];
  }
  sync();
}

// restoration step from the Newton solution: x, s, lambda as in recover_step, p and n
// eliminated (dp = (dlam - r_p)/(Sigma_p + dw), dn = (-dlam - r_n)/(Sigma_n + dw))
__device__ __noinline__ StepInfo recover_step_resto(const Agent a, double mu, double tau, double dw) {
  KState& K = gL.ks;
  const int lane = lane_now();
  const double zeta = K.zeta;
  double amax = 1.0, az = 1.0, gphid = 0.0, theta = 0.0, bar = 0.0;
  for (int i = NX + lane; i < NW; i += WAVE) {
    const double lo = a.xL()[i], hi = a.xU()[i];
    const double sv = gL.u.sol[((i - NX) / NP) * NB + (i - NX) % NP];
    const bool free_ = lo != hi;
    const double d = free_ ? sv : 0.0;
    a.dx()[i] = d;
    if (!free_) continue;
    const double xv = a.x()[i], zl = a.zL()[i], zu = a.zU()[i];
    double gphi = zeta * dr2_of(a.xr()[i]) * (xv - a.xr()[i]);
    if (isfin(lo)) {
      const double s_l = xv - lo;
      gphi -= mu / s_l;
      if (d < 0) amax = fmin(amax, -tau * s_l / d);
      const double dz = mu / s_l - zl - (zl / s_l) * d;
      if (dz < 0) az = fmin(az, -tau * zl / dz);
      bar += log(s_l);
    }
    if (isfin(hi)) {
      const double s_u = hi - xv;
      gphi += mu / s_u;
      if (d > 0) amax = fmin(amax, tau * s_u / d);
      const double dz = mu / s_u - zu + (zu / s_u) * d;
      if (dz < 0) az = fmin(az, -tau * zu / dz);
      bar += log(s_u);
    }
    gphid += gphi * d;
  }
  for (int i = lane; i < NX; i += WAVE) a.dx()[i] = 0.0;
  for (int c = lane; c < M; c += WAVE) {
    const double lbv = a.lb()[c], ubv = a.ub()[c], slo = a.sL()[c], sup = a.sU()[c];
    const double sv = a.s()[c], lm = a.lam()[c], vl = a.vL()[c], vu = a.vU()[c];
    const double gvv = a.gv()[c], gsc = a.gs()[c];
    const double pv = a.rp()[c], nv = a.rn()[c], zp = a.rzp()[c], zn = a.rzn()[c];
    const double dlam = gL.u.sol[(c / NG) * NB + NP + c % NG];
    a.dl()[c] = dlam;
    const int cl = cls_of(lbv, ubv, slo, sup);
    theta += fabs((cl == 0 ? gvv - gsc * lbv : gvv - sv) - pv + nv);
    double dsv = 0.0;
    if (cl == 1) {
      double gphis = 0.0;
      if (isfin(slo)) gphis -= mu / (sv - slo);
      if (isfin(sup)) gphis += mu / (sup - sv);
      const double rs = gphis - lm;
      dsv = (dlam - rs) / (sigma_s_v(sv, slo, sup, vl, vu) + dw);
      gphid += (rs + lm) * dsv;
      if (isfin(slo)) {
        const double s_l = sv - slo;
        if (dsv < 0) amax = fmin(amax, -tau * s_l / dsv);
        const double dv = mu / s_l - vl - (vl / s_l) * dsv;
        if (dv < 0) az = fmin(az, -tau * vl / dv);
        bar += log(s_l);
      }
      if (isfin(sup)) {
        const double s_u = sup - sv;
        if (dsv > 0) amax = fmin(amax, tau * s_u / dsv);
        const double dv = mu / s_u - vu + (vu / s_u) * dsv;
        if (dv < 0) az = fmin(az, -tau * vu / dv);
        bar += log(s_u);
      }
    }
    a.ds()[c] = dsv;
    const double gp = RESTO_RHO - mu / pv, gn = RESTO_RHO - mu / nv;
    const double dp = (dlam - resto_r(-lm, mu / pv)) / (zp / pv + dw);
    const double dn = (-dlam - resto_r(lm, mu / nv)) / (zn / nv + dw);
    a.rdp()[c] = dp;
    a.rdn()[c] = dn;
    gphid += gp * dp + gn * dn;
    if (dp < 0) amax = fmin(amax, -tau * pv / dp);
    if (dn < 0) amax = fmin(amax, -tau * nv / dn);
    const double dzp = mu / pv - zp - (zp / pv) * dp, dzn = mu / nv - zn - (zn / nv) * dn;
    if (dzp < 0) az = fmin(az, -tau * zp / dzp);
    if (dzn < 0) az = fmin(az, -tau * zn / dzn);
    bar += log(pv) + log(nv);
  }
  StepInfo st;
  st.amax = wmin(amax);
  st.az = wmin(az);
  st.gphid = wsum(gphid);
  st.theta = wsum(theta);
  st.barrier = wsum(bar);
  return st;
}

// filter line search of the restoration problem (its own filter in LDS)
__device__ __noinline__ void line_search_resto(const Agent a) {
  KArgs* const argp = kargs();
  KState& K = gL.ks;
  {
    KArgs& ka = *argp;
    const double gphid = K.st.gphid, theta = K.st.theta;
    double amin;
    if (gphid < 0 && theta <= K.theta_min)
      amin = ka.opt.alpha_min_frac * fmin(fmin(ka.opt.gamma_theta, ka.opt.gamma_phi * theta / (-gphid)),
                                     ka.opt.delta * pow_ool(theta, ka.opt.s_theta) / pow_ool(-gphid, ka.opt.s_phi));
    else if (gphid < 0)
      amin = ka.opt.alpha_min_frac * fmin(ka.opt.gamma_theta, ka.opt.gamma_phi * theta / (-gphid));
    else
      amin = ka.opt.alpha_min_frac * ka.opt.gamma_theta;
    if (!(amin > 0.0)) amin = ka.opt.alpha_min_frac * ka.opt.gamma_theta;
    K.amin = amin;
    K.ls.alpha = K.st.amax;
    K.ls.accepted = 0;
    K.ls.ftype = 0;
    K.ls.trials = 0;
    K.ls.tr = Trial{0.0, 0.0, 0.0, 0.0};
    K.ls.bar = 0.0;
    TRACE_LS_HEAD(argp);
  }
#pragma unroll 1
  for (int ls = 0; ls < 64; ++ls) {
    {
      const int lane = lane_now();
      const double alpha = K.ls.alpha;
      double barx = 0.0, prox = 0.0;
#pragma unroll 1
      for (int sl = 0; sl < VS; ++sl) {
        const int i = lane + sl * WAVE;
        if (i < NW) {
          const double lo = a.xL()[i], hi = a.xU()[i];
          const double xt = a.x()[i] + alpha * a.dx()[i];
          gL.u.t.xt[i] = xt;
          if (i >= NX && lo != hi) {
            const double xrv = a.xr()[i];
            prox += dr2_of(xrv) * (xt - xrv) * (xt - xrv);
            if (isfin(lo)) barx += log_ool(xt - lo);
            if (isfin(hi)) barx += log_ool(hi - xt);
          }
        }
      }
      K.barx = wsum(barx);
      K.prox = wsum(prox);
    }
    wsync();
    {
      const double f = eval_fg_lds(a);
      K.ls.tr.f = K.obj_scale * f;
    }
    wsync();
    const int lane = lane_now();
    const double alpha = K.ls.alpha;
    double th = 0.0, bar = 0.0, pn = 0.0;
#pragma unroll 1
    for (int sl = 0; sl < CS; ++sl) {
      const int c = lane + sl * WAVE;
      if (c < M) {
        const double gsv = a.gs()[c], lbv = a.lb()[c], slv = a.sL()[c], suv = a.sU()[c];
        const int cl = cls_of(lbv, a.ub()[c], slv, suv);
        const double gt = gL.u.t.gt[c] * gsv;
        gL.u.t.gt[c] = gt;
        const double st = a.s()[c] + alpha * a.ds()[c];
        const double pt = a.rp()[c] + alpha * a.rdp()[c], nt = a.rn()[c] + alpha * a.rdn()[c];
        th += fabs((cl == 0 ? gt - gsv * lbv : gt - st) - pt + nt);
        if (cl == 1) {
          if (isfin(slv)) bar += log_ool(st - slv);
          if (isfin(suv)) bar += log_ool(suv - st);
        }
        bar += log_ool(pt) + log_ool(nt);
        pn += pt + nt;
      }
    }
    KArgs& ka = *argp;
    const double mu = K.mu, theta = K.st.theta, gphid = K.st.gphid;
    const double phi = K.fx - mu * K.st.barrier;
    Trial tr = K.ls.tr;
    tr.theta = wsum(th);
    tr.fr = RESTO_RHO * wsum(pn) + 0.5 * K.zeta * K.prox;
    tr.phi = tr.fr - mu * (K.barx + wsum(bar));
    K.ls.tr = tr;
    K.ls.trials += 1;
    // a trial whose barrier function is not finite (a slack rounded to 0: phi = +inf) is cut back like
    // an evaluation error (IPOPT BacktrackingLineSearch; oracle/ipm.py rejects it) -- the theta-reduction
    // branch below would otherwise take it and the next iterate's barrier terms are inf / NaN
    bool okt = (tr.theta <= K.theta_max) && isfin(tr.phi);
    {  // filter test, one entry per lane (MAXF <= 64): one LDS read instead of nfilt in sequence
      const int j = lane_now();
      const bool dom = j < K.nfilt && tr.theta >= gL.fth[j < MAXF ? j : 0] && tr.phi >= gL.fph[j < MAXF ? j : 0];
      if (__any(dom)) okt = false;
      if (okt && K.nsp[K.resto] > 0 && spill_dominates(tr.theta, tr.phi)) okt = false;  // older entries
    }
    const bool okf = okt;
    (void)okf;
    bool ftype = false;
    if (okt) {
      const bool switching = gphid < 0 && alpha * pow_ool(-gphid, ka.opt.s_phi) > ka.opt.delta * pow_ool(theta, ka.opt.s_theta);
      if (theta <= K.theta_min && switching) {
        okt = tr.phi <= phi + ka.opt.eta_phi * alpha * gphid;
        ftype = true;
      } else {
        okt = tr.theta <= (1.0 - ka.opt.gamma_theta) * theta || tr.phi <= phi - ka.opt.gamma_phi * theta;
        ftype = false;
      }
    }
    K.ls.ftype = ftype;
    TRACE_LS_TRIAL(argp, alpha, tr, okf, okt, ftype);
    if (okt) { K.ls.accepted = 1; break; }
    if (alpha * 0.5 < K.amin) break;
    K.ls.alpha = alpha * 0.5;
  }
  wsync();
}

// take the restoration trial: accept_step plus p, n and their multipliers
__device__ __noinline__ void accept_step_resto(const Agent a, const double kappa_sigma, double mu, double alpha,
                                               double az) {
  accept_step(a, kappa_sigma, mu, alpha, az);
  const int lane = lane_now();
  for (int c = lane; c < M; c += WAVE) {
    const double pv = a.rp()[c], nv = a.rn()[c], dp = a.rdp()[c], dn = a.rdn()[c];
    const double zp = a.rzp()[c], zn = a.rzn()[c];
    const double pn_ = pv + alpha * dp, nn_ = nv + alpha * dn;
    const double zpn = zp + az * (mu / pv - zp - (zp / pv) * dp);
    const double znn = zn + az * (mu / nv - zn - (zn / nv) * dn);
    a.rp()[c] = pn_;
    a.rn()[c] = nn_;
    a.rzp()[c] = fmax(fmin(zpn, kappa_sigma * mu / pn_), mu / (kappa_sigma * pn_));
    a.rzn()[c] = fmax(fmin(znn, kappa_sigma * mu / nn_), mu / (kappa_sigma * nn_));
  }
}


// filter insertion of the current (theta, phi) with IPOPT's margins
__device__ __forceinline__ void filter_augment(KArgs* argp) {
  KState& K = gL.ks;
  const double gt = (*argp).opt.gamma_theta, gp = (*argp).opt.gamma_phi;
  const double theta = K.st.theta, phi = K.fx - K.mu * K.st.barrier;
  filter_insert((1.0 - gt) * theta, phi - gp * theta);
}

// rest of a restoration iteration after the step: line search, filter, accept.  1: stop
__device__ __noinline__ int resto_tail(const Agent a) {
  KArgs* const argp = kargs();
  KState& K = gL.ks;
  line_search_resto(a);
  const LSResult ls = K.ls;
  K.n_trials += ls.trials;
#ifdef MPCX_TRACE_IT
  if (lane_now() == 0)
    printf("mpcx resto-ls it=%d acc=%d mu=%.6e theta=%.6e phi=%.14e gphid=%.6e amin=%.3e amax=%.3e alpha=%.3e trials=%d "
           "tr.theta=%.6e tr.phi=%.14e thmin=%.3e thmax=%.3e\n", K.it, ls.accepted, K.mu, K.st.theta,
           K.fx - K.mu * K.st.barrier, K.st.gphid, K.amin, K.st.amax, ls.alpha, ls.trials, ls.tr.theta, ls.tr.phi,
           K.theta_min, K.theta_max);
#endif
  if (!ls.accepted) { K.status = MPCX_RESTORATION_FAILED; return 1; }
  if (!ls.ftype) filter_augment(argp);
  K.fx = ls.tr.fr;
  K.fo = ls.tr.f;
  wsync();
  accept_step_resto(a, (*argp).opt.kappa_sigma, K.mu, ls.alpha, K.st.az);
  sync();
  eval_gj_lds(a);
  sync();
  K.it += 1;
  K.n_resto_it += 1;
  return 0;
}

// the step of an original-problem iteration: 0 line-search step, 1 soft step accepted by
// the filter (taken like a line-search step), 2 soft step accepted by the error test
// (already the iterate), -1 restoration phase started, -2 stop at an acceptable point
__device__ MPCX_HOT int search_step(const Agent a) {
  KArgs* const argp = kargs();
  KState& K = gL.ks;
  int mode;
  if (K.soft) {
    K.soft_count += 1;
    const int r = (K.soft_count <= MAX_SOFT_ITERS) ? soft_try(a) : 0;
    if (r == 1) { K.soft = 0; K.soft_count = 0; }
    mode = r == 0 ? -1 : r;
  } else {
    line_search(a);
    K.n_trials += K.ls.trials;
    if (K.ls.accepted) {
      mode = 0;
    } else {
      const int r = soft_try(a);
      if (r != 0) { K.n_soft += 1; if (r == 2) { K.soft = 1; K.soft_count = 0; } }
      mode = r == 0 ? -1 : r;
    }
  }
  if (mode < 0) {
    // "Restoration phase called at acceptable point"
    Acceptable acc = K.acc;
    const OptErr e0 = K.e0;
    const bool acceptable = current_is_acceptable(acc, e0, e0.err_at(0.0), K.fx, K.it, K.obj_scale, K.square,
                                                  (*argp).opt);
    K.acc = acc;
    if (acceptable) { K.status = MPCX_SOLVED_TO_ACCEPTABLE; return -2; }
    resto_start(a);
    return -1;
  }
  return mode;
}

}  // namespace mpcx_kernel

using namespace mpcx_kernel;

// Diagnostic build only (-DMPCX_PROFILE): per-phase shader-clock cycles of each
// agent are written to lam_w[agent][0..15] instead of the bound multipliers.
#ifdef MPCX_PROFILE
#define PROF_DECL unsigned long long _pt = __builtin_amdgcn_s_memtime(); double _prof[16] = {0};
#define PROF(i) do { const unsigned long long _n = __builtin_amdgcn_s_memtime(); _prof[i] += (double)(_n - _pt); _pt = _n; } while (0)
#else
#define PROF_DECL
#define PROF(i) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// the kernel: one agent NLP per workgroup (one wavefront)
// ---------------------------------------------------------------------------
#define KOPT (((KArgs*)__builtin_amdgcn_kernarg_segment_ptr())->opt)
#define OPT(f) (*(volatile const __attribute__((address_space(4))) decltype(mpcx_options::f)*)&KOPT.f)
extern "C" __global__ void __launch_bounds__(64, MIN_WAVES) mpcx_ipm_solve(Args args) {
  // workgroup -> agent: the identity, or the compacted list of the agents still active
  // (mpcx_batch_solve_mapped: a coordinated fleet launches only its unfrozen agents)
  const int agent = args.agent_map != nullptr ? args.agent_map[blockIdx.x] : (int)blockIdx.x;
  if (agent < 0 || agent >= args.n_agents) return;
  if (args.active != nullptr && args.active[agent] == 0) return;  // frozen (converged ADMM block)
  // Loop state lives in LDS (KState, written identically by every lane) and the options are
  // re-read from the kernarg segment where they are used (volatile scalar loads): held in
  // VGPRs they would have to survive every phase call and be spilled to scratch.
  const Agent a{};
  const int lane = lane_now();
  if (lane == 0) {
    gL.kp_bits = (unsigned long long)__builtin_amdgcn_kernarg_segment_ptr();
    gL.ws_bits = (unsigned long long)((gdbl*)args.ws + (long)agent * args.ws_stride);
#ifdef MPCX_TRACE_LS
    gL.trace_agent = agent;
#endif
  }
  wsync();
  KState& K = gL.ks;

  PROF_DECL
#ifdef MPCX_PROFILE
  if (lane < 10) gL.sprof[lane] = 0.0;
  if (lane < 2) gL.dense_seen[lane] = 0u;
  sync();
#endif
  if (lane == 0) { gL.want_sdh = 0; gL.sdh_ok = 0; gL.hsig = 1.0; gL.seq = 0; }
  {
    const Scal sc = init_agent(a, agent);
    K.obj_scale = sc.obj_scale;
    K.fx = sc.fx;
    K.square = sc.square;
  }
  K.n_fact = 0; K.n_ic = 0; K.n_fallback = 0; K.n_trials = 0; K.n_chain = 0; K.n_dense = 0;
  PROF(0);
  if (M > 0 && OPT(constr_mult_init_max) > 0.0) {
    ls_mult_rhs(a, K.obj_scale);
    const Inertia in = factor(a, KKTDiag{0.0, 0.0, LSQ});
    if (in.zero == 0) {
      solve(a);
      ls_mult_finish(a, OPT(constr_mult_init_max));
    }
    K.n_fact = 1;
  }
  PROF(1);

  K.mu = OPT(mu_init);
  K.tau = fmax(OPT(tau_min), 1.0 - K.mu);
  K.dw_last = 0.0;
  {
    const double theta0 = theta_now(a);
    K.theta_max = OPT(theta_max_fact) * fmax(1.0, theta0);
    K.theta_min = OPT(theta_min_fact) * fmax(1.0, theta0);
  }
  K.nfilt = 0;
  K.nsp[0] = 0; K.nsp[1] = 0;
  K.status = MPCX_MAX_ITER_EXCEEDED;
  K.it = 0;
  K.acc = Acceptable{-1e50, -1e50, -1, 0};
  K.resto = 0; K.soft = 0; K.soft_count = 0; K.lsmode = 0; K.n_soft = 0; K.n_resto_it = 0;
  K.n_filt_over = 0; K.n_refine = 0;
  K.bar_ok = 0; K.bar_val = 0.0;
#define KARGP ((KArgs*)__builtin_amdgcn_kernarg_segment_ptr())
#pragma unroll 1
  for (;;) {
#ifdef MPCX_TRACE_IT  // diagnostics (scripts/resto_ab.py trace): the previous iteration's step, per iteration
    {
      double mxl = INFINITY;
      int arg = -1;
      for (int i = NX + lane; i < NW; i += WAVE) {
        const double lo = a.xL()[i];
        if (lo != a.xU()[i] && isfin(lo) && a.x()[i] - lo < mxl) { mxl = a.x()[i] - lo; arg = i; }
      }
      const double m = wmin(mxl);
      const int am = (int)wmax(mxl == m ? (double)arg : -1.0);
      if (lane == 0 && agent == 0)
        printf("mpcx it=%d resto=%d soft=%d mu=%.6e fx=%.14e theta=%.6e amax=%.3e alpha=%.4e trials=%d refine=%d dw=%.3e "
               "nfilt=%d min x-lo=%.3e at %d\n", K.it, K.resto, K.soft, K.mu, K.fx, K.st.theta, K.st.amax, K.ls.alpha,
               K.ls.trials, K.n_refine, K.dw, K.nfilt, m, am);
    }
#endif
    if (K.resto) {
      const int hr = iter_head_resto(a);
      if (hr == 1) break;
      if (hr == 2) resto_return(a);  // back in the original problem: its own head at this point
    }
    if (!K.resto && iter_head(a)) break;  // one (inlined) call site
    PROF(2);
    eval_hess(a, K.resto ? 0.0 : K.obj_scale);  // restoration: the constraints' curvature only
    PROF(3);
    // factorisation with inertia correction (IPOPT Algorithm IC); in the restoration phase the
    // same loop then re-factors for the iterative-refinement corrections (one factor() call
    // site: it is inlined into the kernel body)
    K.dw = 0.0;
    K.dc = 0.0;
    int ok = 0, refining = 0, steps = 0;
    double old_ratio = 0.0;
#pragma unroll 1
    for (int attempt = 0; attempt < IC_ATTEMPTS + MAX_REFINE + 2; ++attempt) {
      if (!refining && attempt >= IC_ATTEMPTS) break;
      if (attempt > 0 && !refining) {  // attempt 0: the iteration head wrote the rhs
        if (K.resto) rhs_dual_resto(a, K.mu, K.dw, K.dc);
        else rhs_dual(a, K.mu, K.dw, K.dc);
      }
      const Inertia in = factor(a, KKTDiag{K.dw, K.dc, NEWTON});
#ifdef MPCX_TRACE_IC  // diagnostics: long inertia-correction sequences
      if (!refining && attempt > 2 && lane_now() == 0)
        printf("mpcx ic it=%d resto=%d att=%d dw=%.3e dc=%.3e mu=%.3e pos=%d neg=%d zero=%d want=%d/%d\n", K.it,
               K.resto, attempt, K.dw, K.dc, K.mu, in.pos, in.neg, in.zero, N * NP, M);
#endif
      if (refining) {  // correction for the residual in the rhs: add it, re-test
        solve(a);
        resto_step_io(a, 1);
        steps += 1;
        const double ratio = resto_resid(a, 0);
        if (ratio <= RESID_RATIO_MAX && steps >= MIN_REFINE) break;
        if (steps > MIN_REFINE && (steps > MAX_REFINE || ratio > RESID_IMPROVE * old_ratio)) break;
        old_ratio = ratio;
        resto_step_io(a, 0);
        continue;
      }
      K.n_fact += 1;
      K.n_chain += gL.seq;
      if (in.pos == N * NP && in.neg == M && in.zero == 0) {
        if (attempt > 0) K.dw_last = K.dw;
        ok = 1;
        if (!K.resto) break;
        solve(a);
        old_ratio = resto_resid(a, 1);
        if (MIN_REFINE == 0 && old_ratio <= RESID_RATIO_MAX) break;
        refining = 1;
        resto_step_io(a, 0);
        continue;
      }
      K.n_ic += 1;
      const double dw = K.dw, dw_last = K.dw_last;
      if (attempt == 0) {
        if (in.zero > 0) K.dc = OPT(delta_c_bar) * pow_ool(K.mu, OPT(kappa_c));
        K.dw = (dw_last == 0.0) ? OPT(delta_w_first) : fmax(OPT(delta_w_min), OPT(kappa_w_minus) * dw_last);
      } else {
        K.dw = (dw_last == 0.0) ? OPT(kappa_w_plus_bar) * dw : OPT(kappa_w_plus) * dw;
        if (K.dw > OPT(delta_w_max)) {
          // IPOPT PDPerturbationHandler::PerturbForWrongInertia: the Hessian shift alone cannot
          // fix the inertia (a constraint direction the Jacobian does not span) -- regularise the
          // constraint block as for a singular matrix and run the shifts again from the start
          if (K.dc != 0.0) break;
          K.dc = OPT(delta_c_bar) * pow_ool(K.mu, OPT(kappa_c));
          K.dw = (dw_last == 0.0) ? OPT(delta_w_first) : fmax(OPT(delta_w_min), OPT(kappa_w_minus) * dw_last);
        }
      }
    }
    PROF(5);
    if (!ok) { K.status = MPCX_ERROR_IN_STEP; break; }
    if (refining) K.n_refine += steps;
    else solve(a);
    PROF(6);
    if (K.resto) {
      const StepInfo st = recover_step_resto(a, K.mu, K.tau, K.dw);
      K.st = st;
    } else {
#ifndef MPCX_NO_BARCACHE
      const StepInfo st = recover_step(a, K.mu, K.tau, K.dw, K.obj_scale, K.bar_ok);
#else  // diagnostics (A/B): the barrier recomputed at every iterate
      const StepInfo st = recover_step(a, K.mu, K.tau, K.dw, K.obj_scale, 0);
#endif
      K.st = st;
    }
    PROF(7);
    if (K.resto) {  // restoration iteration: its own filter; no restoration inside it
      if (resto_tail(a)) break;
      continue;
    }
    // filter line search; on failure the soft restoration step, then the restoration phase
    // (IPOPT BacktrackingLineSearch::FindAcceptableTrialPoint)
    const int mode = search_step(a);
    K.bar_ok = 0;                // the iterate changes below; only an accepted trial re-validates it
    if (mode == -2) break;       // acceptable point, status set
    if (mode == -1) continue;    // restoration phase started
    if (mode == 2) {  // the soft trial is already the iterate
      K.fx = K.ls.tr.f;
      wsync();
      K.it += 1;
      continue;
    }
    if (!K.ls.ftype) filter_augment(KARGP);
    K.fx = K.ls.tr.f;
    wsync();
    PROF(8);
    accept_step(a, OPT(kappa_sigma), K.mu, K.ls.alpha, mode == 1 ? K.ls.alpha : K.st.az);
    K.bar_val = K.ls.bar;        // the new iterate IS the last trial point: its barrier sum holds
    K.bar_ok = 1;
    sync();  // accepted multipliers visible to the stage lanes
    eval_gj_lds(a);
    sync();
    K.it += 1;
    PROF(9);
  }
#undef KARGP
#ifdef MPCX_TRACE_IT
  if (lane == 0 && agent == 0) printf("mpcx end it=%d resto=%d status=%d\n", K.it, K.resto, K.status);
#endif
  const double obj_scale = K.obj_scale;

  // ---- outputs ----------------------------------------------------------------
  gdbl* wio = (gdbl*)args.w + (long)agent * NW;
  // stopped inside the restoration phase: the original problem's objective and bound
  // multipliers (those at the start of restoration), constraint multipliers zero
  const int in_resto = K.resto;
  for (int i = lane; i < NW; i += WAVE) {
    wio[i] = a.x()[i];
#ifndef MPCX_TRACE_LS
    if (args.lam_w != nullptr)
#else
    if (false)
#endif
      ((gdbl*)args.lam_w)[(long)agent * NW + i] =
          (i < NX) ? 0.0 : (in_resto ? a.zu0()[i] - a.zl0()[i] : a.zU()[i] - a.zL()[i]) / obj_scale;
  }
#ifdef MPCX_PROFILE
  PROF(2);
  for (int i = 0; i < 6; ++i) _prof[10 + i] = gL.sprof[i];
  sync();
  if (args.lam_w != nullptr && lane == 0)
    for (int i = 0; i < 16 && i < NW; ++i) ((gdbl*)args.lam_w)[(long)agent * NW + i] = _prof[i];
  if (args.lam_w != nullptr && lane == 0 && NW > 17) {
    ((gdbl*)args.lam_w)[(long)agent * NW + 16] = (double)gL.dense_seen[0];
    ((gdbl*)args.lam_w)[(long)agent * NW + 17] = (double)gL.dense_seen[1];
  }
  if (args.lam_w != nullptr && lane == 0 && NW > 21)
    for (int i = 6; i < 10; ++i) ((gdbl*)args.lam_w)[(long)agent * NW + 12 + i] = gL.sprof[i];
#endif
#ifndef MPCX_TRACE_LS
  if (args.lam_g != nullptr)
#else
  if (false)
#endif
    for (int c = lane; c < M; c += WAVE)
      ((gdbl*)args.lam_g)[(long)agent * M + c] = in_resto ? 0.0 : a.lam()[c] * a.gs()[c] / obj_scale;
  if (args.stats != nullptr && lane == 0) {
    mpcx_stats st;
    st.obj = (in_resto ? K.fo : K.fx) / obj_scale;
    st.primal_inf = K.e0.viol_u;
    st.dual_inf = K.e0.dual_u;
    st.compl_inf = K.e0.compl_at(0.0) / obj_scale;
    st.mu = K.mu;
    st.obj_scale = obj_scale;
    st.iter_count = K.it;
    st.status = K.status;
    st.n_inertia_corrections = K.n_ic;
    st.n_restorations = K.n_fallback;
    st.n_soft_restorations = K.n_soft;
    st.n_restoration_iters = K.n_resto_it;
    st.n_filter_overflows = K.n_filt_over;
    st.n_refinement_steps = K.n_refine;
    st.n_factorizations = K.n_fact;
    st.n_trials = K.n_trials;
    st.n_block_chain = K.n_chain;
    st.n_dense_stages = K.n_dense;
    args.stats[agent] = st;
  }
}

extern "C" __global__ void mpcx_query(long* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = WS_DOUBLES;
    out[1] = N; out[2] = NX; out[3] = NV; out[4] = NG; out[5] = NPS; out[6] = NPG;
    out[7] = MPCX_KERNEL_ABI;  // one definition (mpcx_internal.h), checked by mpcx_problem_create
    out[8] = sizeof(Lds);
#ifdef MPCX_WS_LDS
    out[9] = 1;  // workspace in LDS: one agent per CU (small fleets)
#else
    out[9] = 0;
#endif
    out[10] = MIN_WAVES;  // waves per SIMD the register budget is compiled for
    out[11] = APC;        // agents per CU the LDS share allows
  }
}
