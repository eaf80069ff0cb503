// Developer micro-benchmark (not product code): cycles per step of an 11-vector recursion
// pv_{k} = M pv_{k+1} + v on one wave, with the cross-lane broadcast done four ways.
// Build: hipcc --offload-arch=gfx950 -O3 chain_ubench.hip -o chain_ubench; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NX = 11, STEPS = 2048;

__device__ __forceinline__ float rl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }

template <int MODE>
__global__ void chain(const float* m, float* out, long long* cyc) {
  __shared__ float sh[64 * 4];
  const int ln = threadIdx.x;
  float mr[NX];
  for (int j = 0; j < NX; ++j) mr[j] = m[ln * NX + j] * 0.01f;
  float v = m[ln] * 0.1f;
  float pv = m[ln + 64];
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < STEPS; ++s) {
    float p[NX];
    if (MODE == 0 || MODE == 1) {
      for (int j = 0; j < NX; ++j) p[j] = rl(pv, j);
    } else if (MODE == 2) {  // LDS broadcast
      sh[ln] = pv;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int j = 0; j < NX; ++j) p[j] = sh[j];
    } else {  // ds_bpermute (shfl) per element
      for (int j = 0; j < NX; ++j) p[j] = __shfl(pv, j, 64);
    }
    float a;
    if (MODE == 0) {
      a = v;
      for (int j = 0; j < NX; ++j) a += mr[j] * p[j];
    } else {
      float a0 = v + mr[0] * p[0], a1 = mr[1] * p[1], a2 = mr[2] * p[2];
      for (int j = 3; j < NX; j += 3) {
        a0 += mr[j] * p[j];
        if (j + 1 < NX) a1 += mr[j + 1] * p[j + 1];
        if (j + 2 < NX) a2 += mr[j + 2] * p[j + 2];
      }
      a = (a0 + a1) + a2;
    }
    pv = a;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[ln] = pv;
  if (ln == 0) cyc[0] = t1 - t0;
}

int main() {
  float *m, *out;
  long long* cyc;
  hipMalloc(&m, 64 * NX * 4 * sizeof(float));
  hipMalloc(&out, 64 * sizeof(float));
  hipMalloc(&cyc, sizeof(long long));
  float hm[64 * NX * 4];
  for (int i = 0; i < 64 * NX * 4; ++i) hm[i] = (float)((i * 37) % 101) / 101.0f;
  hipMemcpy(m, hm, sizeof(hm), hipMemcpyHostToDevice);
  const char* names[4] = {"readlane+serial dot", "readlane+3-chain dot", "LDS broadcast+3-chain", "bpermute+3-chain"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 4; ++mode) {
      if (mode == 0) hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, m, out, cyc);
      if (mode == 1) hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, m, out, cyc);
      if (mode == 2) hipLaunchKernelGGL(chain<2>, dim3(1), dim3(64), 0, 0, m, out, cyc);
      if (mode == 3) hipLaunchKernelGGL(chain<3>, dim3(1), dim3(64), 0, 0, m, out, cyc);
      long long c;
      hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
      if (rep) printf("%-26s %7.1f cycles/step (s_memtime ticks)\n", names[mode], (double)c / STEPS);
    }
  return 0;
}
