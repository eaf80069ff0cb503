// Developer check (not product code): accuracy and dependent-chain latency of the fp64 reciprocal square root
// of the Riccati pivots (mr_common.h mr_rsqrt: v_rsq_f64 + two Newton steps) against the library's 1.0 / sqrt.
// Prints the largest error in ulps of the IEEE value over 2^22 log-uniform inputs in [1e-30, 1e40] and the
// cycles per dependent evaluation of each form.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ double rsq_newton(double a) {
  double y = __builtin_amdgcn_rsq(a);
#pragma unroll
  for (int i = 0; i < 2; ++i) y = __builtin_fma(0.5 * y, __builtin_fma(-(a * y), y, 1.0), y);
  return y;
}
__device__ __forceinline__ double rsq_lib(double a) { return 1.0 / sqrt(a); }

__global__ void err(const double* x, double* worst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double r = rsq_lib(x[i]), f = rsq_newton(x[i]);
  const double ulp = ldexp(1.0, ilogb(r) - 52);
  worst[i] = fabs(f - r) / ulp;
}

template <int FORM>
__global__ void chain(double a0, double* out, long long* cyc) {
  double a = a0 + threadIdx.x * 1e-3;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < 1024; ++k) a = 1.5 + (FORM ? rsq_newton(a) : rsq_lib(a));  // dependent chain
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  const int n = 1 << 22;
  double *x, *w, *o;
  long long* c;
  hipMalloc(&x, n * sizeof(double));
  hipMalloc(&w, n * sizeof(double));
  hipMalloc(&o, 64 * sizeof(double));
  hipMalloc(&c, sizeof(long long));
  double* h = new double[n];
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = pow(10.0, -30.0 + 70.0 * (double)(s >> 11) / 9007199254740992.0);
  }
  hipMemcpy(x, h, n * sizeof(double), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(err, dim3(n / 256), dim3(256), 0, 0, x, w, n);
  hipMemcpy(h, w, n * sizeof(double), hipMemcpyDeviceToHost);
  double worst = 0.0;
  int over1 = 0;
  for (int i = 0; i < n; ++i) { worst = fmax(worst, h[i]); over1 += h[i] > 1.0; }
  printf("rsq_newton vs 1/sqrt: max error %.3f ulp, %d of %d inputs above 1 ulp\n", worst, over1, n);
  long long cyc;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, 2.0, o, c);
    hipMemcpy(&cyc, c, sizeof(cyc), hipMemcpyDeviceToHost);
    if (rep) printf("1.0 / sqrt : %.1f cycles per dependent evaluation\n", cyc / 1024.0);
    hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, 2.0, o, c);
    hipMemcpy(&cyc, c, sizeof(cyc), hipMemcpyDeviceToHost);
    if (rep) printf("rsq+Newton : %.1f cycles per dependent evaluation\n", cyc / 1024.0);
  }
  return 0;
}
