// Developer micro-benchmark (not product code): the 11-vector recursion of chain_ubench.hip with
// NLOAD per-step operand loads (global, issued AHEAD steps early, rotating register sets) -- how
// much the loads' issue and the vmcnt waits add to the v_readlane + FMA chain.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NX = 11, STEPS = 1024, STRIDE = 304;

__device__ __forceinline__ float rl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }

template <int NLOAD>
struct Ops { float m[NLOAD]; };

template <int NLOAD>
__device__ __forceinline__ void ld(const float* __restrict__ rec, int k, int ln, Ops<NLOAD>& o) {
  const float* r = rec + (size_t)k * STRIDE;
#pragma unroll
  for (int j = 0; j < NLOAD; ++j) o.m[j] = r[(ln * 7 + j * 13) % STRIDE];
}

template <int NLOAD>
__device__ __forceinline__ float step(float pv, float v, const Ops<NLOAD>& o) {
  float p[NX];
#pragma unroll
  for (int j = 0; j < NX; ++j) p[j] = rl(pv, j);
  float a0 = v + o.m[0 % NLOAD] * p[0], a1 = o.m[1 % NLOAD] * p[1], a2 = o.m[2 % NLOAD] * p[2];
#pragma unroll
  for (int j = 3; j < NX; j += 3) {
    a0 += o.m[j % NLOAD] * p[j];
    if (j + 1 < NX) a1 += o.m[(j + 1) % NLOAD] * p[j + 1];
    if (j + 2 < NX) a2 += o.m[(j + 2) % NLOAD] * p[j + 2];
  }
  float extra = 0.f;
#pragma unroll
  for (int j = NX; j < NLOAD; ++j) extra += o.m[j];
  return (a0 + a1) + a2 + 1e-9f * extra;
}

template <int NLOAD>
__global__ void chain(const float* rec, float* out, long long* cyc) {
  const int ln = threadIdx.x;
  float v = rec[ln] * 0.1f;
  float pv = rec[ln + 64];
  Ops<NLOAD> b0, b1, b2, b3;
  ld(rec, 0, ln, b0); ld(rec, 1, ln, b1); ld(rec, 2, ln, b2);
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < STEPS; k += 4) {
    ld(rec, k + 3, ln, b3);
    __builtin_amdgcn_sched_barrier(0);
    pv = step(pv, v, b0);
    ld(rec, k + 4, ln, b0);
    __builtin_amdgcn_sched_barrier(0);
    pv = step(pv, v, b1);
    ld(rec, k + 5, ln, b1);
    __builtin_amdgcn_sched_barrier(0);
    pv = step(pv, v, b2);
    ld(rec, k + 6, ln, b2);
    __builtin_amdgcn_sched_barrier(0);
    pv = step(pv, v, b3);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[ln] = pv;
  if (ln == 0) cyc[0] = t1 - t0;
}

int main() {
  float *rec, *out;
  long long* cyc;
  const size_t n = (size_t)(STEPS + 8) * STRIDE;
  hipMalloc(&rec, n * sizeof(float));
  hipMalloc(&out, 64 * sizeof(float));
  hipMalloc(&cyc, sizeof(long long));
  float* h = new float[n];
  for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 37) % 101) / 1010.0f;
  hipMemcpy(rec, h, n * sizeof(float), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    long long c;
#define RUN(NL)                                                                   \
    hipLaunchKernelGGL(chain<NL>, dim3(1), dim3(64), 0, 0, rec, out, cyc);        \
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);                          \
    if (rep) printf("loads/step %2d: %7.1f cycles/step\n", NL, (double)c / STEPS);
    RUN(1) RUN(6) RUN(11) RUN(17) RUN(23)
  }
  return 0;
}
