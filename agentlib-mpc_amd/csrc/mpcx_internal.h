// mpcx_internal.h — layout shared by the host runtime (mpcx_runtime.cpp) and
// the generated IPM code objects (mpcx_ipm.hip).  Not part of the public ABI.
#ifndef MPCX_INTERNAL_H
#define MPCX_INTERNAL_H

#include "mpcx.h"

#define MPCX_KERNEL_ABI 8

typedef struct mpcx_kernel_args {
  const double* p;
  const double* lbw;
  const double* ubw;
  const double* lbg;
  const double* ubg;
  double* w;
  double* lam_g;
  double* lam_w;
  mpcx_stats* stats;
  const int* active;
  const int* agent_map;  // workgroup -> agent (mpcx_batch_solve_mapped; -1: no agent), or NULL
  double* ws;
  long ws_stride;
  int n_agents;
  int pad;
  mpcx_options opt;
} mpcx_kernel_args;

#endif
