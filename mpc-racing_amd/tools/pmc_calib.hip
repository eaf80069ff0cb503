// PMC calibration (developer tool, not the product): FETCH_SIZE / WRITE_SIZE against known byte counts
// for the access widths the solve kernel uses (4-byte and 8-byte per lane buffer loads / stores), as the
// MI355X guide asks before trusting absolutes ("other access widths are uncalibrated").
//
//   hipcc --offload-arch=gfx950 -O3 -o variants/pmc_calib mpc-racing_amd/tools/pmc_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -- variants/pmc_calib ;  rocprofv3 --pmc WRITE_SIZE -- variants/pmc_calib
//
// Each kernel touches a 1 GiB buffer once (4x the 256 MiB MALL, so nothing is served on-die from an
// earlier pass), 256-lane workgroups, consecutive lanes on consecutive words (coalesced).
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr size_t kBytes = size_t(1) << 30;

__global__ __launch_bounds__(256) void rd4(const float* a, float* out, size_t n) {
  float s = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) s += a[i];
  if (s == 12345.f) out[threadIdx.x] = s;  // keeps the loads (never true for the zero-filled input)
}
__global__ __launch_bounds__(256) void wr4(float* a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) a[i] = 1.f;
}
__global__ __launch_bounds__(256) void rd8(const double* a, double* out, size_t n) {
  double s = 0.0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) s += a[i];
  if (s == 12345.0) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void wr8(double* a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) a[i] = 1.0;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  void *a, *b, *out;
  CK(hipMalloc(&a, kBytes));
  CK(hipMalloc(&b, kBytes));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(a, 0, kBytes));
  CK(hipMemset(b, 0, kBytes));
  const dim3 g(8192), t(256);
  hipLaunchKernelGGL(rd4, g, t, 0, 0, (const float*)a, (float*)out, kBytes / 4);
  hipLaunchKernelGGL(wr4, g, t, 0, 0, (float*)b, kBytes / 4);
  hipLaunchKernelGGL(rd8, g, t, 0, 0, (const double*)b, (double*)out, kBytes / 8);
  hipLaunchKernelGGL(wr8, g, t, 0, 0, (double*)a, kBytes / 8);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("{\"bytes_per_kernel\": %zu, \"kernels\": [\"rd4\", \"wr4\", \"rd8\", \"wr8\"]}\n", kBytes);
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(out));
  return 0;
}
