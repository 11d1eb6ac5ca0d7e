// FETCH_SIZE / WRITE_SIZE calibration on known byte counts (the guide calibrates
// FETCH_SIZE only for 16-B/lane streaming reads; the IPM kernel mostly issues 8-B/lane loads).
//
// Each kernel streams a 1 GiB buffer once (4x the 256 MiB Infinity Cache: every line comes from
// HBM) with one access width, coalesced (lane i of a wave-instruction at element i: 64 lanes x
// width contiguous bytes -- the IPM kernel's vector-phase pattern, one element per lane):
//   read4 / read8 / read16   global_load_dword / _dwordx2 / _dwordx4, one per lane per step
//   write8 / write16         global_store_dwordx2 / _dwordx4
//   read8_agent              8-B loads in the IPM's shape: one 64-lane workgroup per "agent", each
//                            reading its own contiguous slab (97 KB, the C3 workspace) front to back
// rocprofv3 --pmc FETCH_SIZE (resp. WRITE_SIZE) then reports per dispatch what the counter says for
// 1 GiB (read8_agent: the slabs' bytes).  usage: fetch_calib [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

__device__ __forceinline__ double val(float v) { return v; }
__device__ __forceinline__ double val(double v) { return v; }
__device__ __forceinline__ double val(double2 v) { return v.x + v.y; }

template <typename T>
__global__ void __launch_bounds__(256) read_k(const T* __restrict__ a, long n, double* __restrict__ out) {
  double s = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    s += val(a[i]);
  }
  if (s == 12345.678) out[blockIdx.x] = s;  // never true for the zero-filled buffer: keeps the loads
}

template <typename T>
__global__ void __launch_bounds__(256) write_k(T* __restrict__ a, long n) {
  T v;
  __builtin_memset(&v, 0, sizeof(T));
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) a[i] = v;
}

// one agent per 64-lane workgroup, its slab of `slab` doubles read front to back, 8 B per lane
__global__ void __launch_bounds__(64) read8_agent(const double* __restrict__ a, long slab, int agents,
                                                  double* __restrict__ out) {
  double s = 0.0;
  for (int ag = blockIdx.x; ag < agents; ag += gridDim.x) {
    const double* p = a + (long)ag * slab;
    for (long i = threadIdx.x; i < slab; i += 64) s += p[i];
  }
  if (s == 12345.678) out[blockIdx.x] = s;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  const size_t bytes = 1ull << 30;
  char* buf = nullptr;
  double* out = nullptr;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, 1 << 20));
  CHECK(hipMemset(buf, 0, bytes));
  const int grid = 256 * 8, block = 256;
  const long slab = 12082;  // doubles per C3 agent workspace
  const int agents = (int)(bytes / (slab * 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < reps; ++r) {
    float ms[6];
    CHECK(hipEventRecord(e0));
    read_k<float><<<grid, block>>>((const float*)buf, (long)(bytes / 4), out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms[0], e0, e1));
    CHECK(hipEventRecord(e0));
    read_k<double><<<grid, block>>>((const double*)buf, (long)(bytes / 8), out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms[1], e0, e1));
    CHECK(hipEventRecord(e0));
    read_k<double2><<<grid, block>>>((const double2*)buf, (long)(bytes / 16), out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms[2], e0, e1));
    CHECK(hipEventRecord(e0));
    write_k<double><<<grid, block>>>((double*)buf, (long)(bytes / 8));
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms[3], e0, e1));
    CHECK(hipEventRecord(e0));
    write_k<double2><<<grid, block>>>((double2*)buf, (long)(bytes / 16));
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms[4], e0, e1));
    CHECK(hipEventRecord(e0));
    read8_agent<<<4096, 64>>>((const double*)buf, slab, agents, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms[5], e0, e1));
    std::printf("rep %d: read4 %.3f ms, read8 %.3f, read16 %.3f, write8 %.3f, write16 %.3f, read8_agent %.3f "
                "(%ld agents x %ld B = %ld bytes)\n",
                r, ms[0], ms[1], ms[2], ms[3], ms[4], ms[5], (long)agents, slab * 8, (long)agents * slab * 8);
  }
  std::printf("bytes per streaming kernel: %zu\n", bytes);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
