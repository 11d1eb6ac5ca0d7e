// mpcx_net_mfma.h — wave-level evaluation of the NARX networks on the FP64 matrix cores.
//
// Included by generated model sources that contain network nodes (runtime/codegen.py,
// device-only section).  What it replaces: the CasADi evaluation of the reference's
// serialized ANN (agentlib_mpc/models/casadi_predictor.py:306-336, one dense hidden layer,
// topology from modules/ml_model_training/ml_model_trainer.py:617-626) inside every IPOPT
// callback.  The per-stage generated code evaluates each network once per stage in a
// loop over the hidden units, one stage per lane (12 of 64 lanes busy for a C5 zone);
// here all evaluations of one network in the agent (stages x call sites, R rows) are one
// batched product per wavefront:
//
//   A^T = W1^T X^T + b1          [H x R]   (v_mfma_f64_16x16x4_f64, K = inputs)
//   v   = w2 . act(A) + b2       [R]       (row sums of the accumulator tile)
//   g^T = W1_D (w2 o act'(A))    [ND1 x R] (K = hidden units)
//   h^T = P_D  (w2 o act''(A))   [ND2 x R] (P_D[p][j] = W1[a_p][j] W1[b_p][j])
//
// Orientation: the first product is computed transposed (hidden unit on the accumulator
// row, evaluation on the lane), so its accumulator register r of lane l holds hidden
// unit 4r + (l >> 4) of evaluation l & 15 -- exactly the B operand of the k-step over
// hidden units 4r .. 4r + 3 of the two derivative products: no LDS round trip and no
// lane movement between the three products.
//
// f64 MFMA lane maps (CDNA4): A[m = l & 15][k = l >> 4], B[k = l >> 4][n = l & 15],
// D lane l register r: [m = (l >> 4) + 4 r][n = l & 15].
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace mpcx_net {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) double ldsd;

// activation codes follow symbolic._ACTS: sigmoid, tanh, linear, softplus, exponential, gaussian
template <int ACT>
__device__ __forceinline__ void act(double a, double& s0, double& s1, double& s2) {
  if constexpr (ACT == 0) {
    s0 = 1.0 / (1.0 + exp(-a)); s1 = s0 * (1.0 - s0); s2 = s1 * (1.0 - 2.0 * s0);
  } else if constexpr (ACT == 1) {
    s0 = tanh(a); s1 = 1.0 - s0 * s0; s2 = -2.0 * s0 * s1;
  } else if constexpr (ACT == 2) {
    s0 = a; s1 = 1.0; s2 = 0.0;
  } else if constexpr (ACT == 3) {
    const double sg = 1.0 / (1.0 + exp(-a));
    s0 = log(1.0 + exp(a)); s1 = sg; s2 = sg * (1.0 - sg);
  } else if constexpr (ACT == 4) {
    s0 = exp(a); s1 = s0; s2 = s0;
  } else {
    s0 = exp(-a * a); s1 = -2.0 * a * s0; s2 = (4.0 * a * a - 2.0) * s0;
  }
}

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// R evaluations of one network (inputs X[R][NIN], LDS) -> V[R] (if WV), G[R][ND1]
// (d/d inputs D1[]), Hd[R][ND2] (d2 / d inputs of pair p, table PW[ND2][H]).  Called by
// all 64 lanes of the wave; every lane takes part in every product.
template <int R, int NIN, int H, int ACT, bool WV, int ND1, int ND2>
__device__ __forceinline__ void eval(const ldsd* X, ldsd* V, ldsd* Gd, ldsd* Hd, const double* W1T,
                                     const double* B1, const double* W2, double b2, const int* D1,
                                     const double* PW, int lane) {
  constexpr int JT = (H + 15) / 16;   // hidden-unit tiles
  constexpr int KS = (NIN + 3) / 4;   // k-steps over the inputs
  constexpr bool W1D = ND1 > 0, W2D = ND2 > 0;
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll 1
  for (int rt = 0; rt < (R + 15) / 16; ++rt) {
    const int row = rt * 16 + lr;
    d4 acc[JT];
#pragma unroll
    for (int jt = 0; jt < JT; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = jt * 16 + lk + 4 * r;
        acc[jt][r] = j < H ? B1[j] : 0.0;
      }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int i = ks * 4 + lk;
      const double bx = (row < R && i < NIN) ? X[row * NIN + i] : 0.0;
#pragma unroll
      for (int jt = 0; jt < JT; ++jt) {
        const int jj = jt * 16 + lr;
        const double aw = (jj < H && i < NIN) ? W1T[jj * NIN + i] : 0.0;
        acc[jt] = mfma(aw, bx, acc[jt]);
      }
    }
    // activations, weighted by the output layer; registers keep the accumulator layout
    double c0[JT][4], c1[JT][4], c2[JT][4];
#pragma unroll
    for (int jt = 0; jt < JT; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = jt * 16 + lk + 4 * r;
        const double w = j < H ? W2[j] : 0.0;
        double s0, s1, s2;
        act<ACT>(acc[jt][r], s0, s1, s2);
        c0[jt][r] = w * s0; c1[jt][r] = w * s1; c2[jt][r] = w * s2;
      }
    if constexpr (WV) {
      double v = 0.0;
#pragma unroll
      for (int jt = 0; jt < JT; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) v += c0[jt][r];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lk == 0 && row < R) V[row] = v + b2;
    }
    if constexpr (W1D) {
#pragma unroll
      for (int it = 0; it < (ND1 + 15) / 16; ++it) {
        const int ii = it * 16 + lr;
        const int col = ii < ND1 ? D1[ii] : 0;
        d4 g = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int jt = 0; jt < JT; ++jt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = jt * 16 + 4 * r + lk;
            const double aw = (ii < ND1 && j < H) ? W1T[j * NIN + col] : 0.0;
            g = mfma(aw, c1[jt][r], g);
          }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int o = it * 16 + lk + 4 * r;
          if (o < ND1 && row < R) Gd[row * ND1 + o] = g[r];
        }
      }
    }
    if constexpr (W2D) {
#pragma unroll
      for (int pt = 0; pt < (ND2 + 15) / 16; ++pt) {
        const int pp = pt * 16 + lr;
        d4 h = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int jt = 0; jt < JT; ++jt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = jt * 16 + 4 * r + lk;
            const double aw = (pp < ND2 && j < H) ? PW[pp * H + j] : 0.0;
            h = mfma(aw, c2[jt][r], h);
          }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int o = pt * 16 + lk + 4 * r;
          if (o < ND2 && row < R) Hd[row * ND2 + o] = h[r];
        }
      }
    }
  }
}

}  // namespace mpcx_net
