// libmpcracing.so -- gfx950 batched racing-MPC solver and its C ABI (include/mpcracing.h).
//
// One 64-lane wavefront per MPC instance runs the interior-point solve (mr_wave.h):
// lanes = stages for the stage-parallel sweeps, lanes = matrix rows for the Riccati
// recursion.  Instances are independent: no inter-workgroup communication.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <string>

#include "mr_wave.h"

using namespace mr;

struct mr_handle {
  mr_config cfg;
  void* ws;
  size_t ws_bytes;
  TyreCoef<double> tf, tr;
  int have_tyres;
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(x)                                                                  \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) return fail(MR_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// One 64-lane workgroup (= one wavefront) per instance: lanes are stages / matrix rows
// of that instance (mr_wave.h); the grid is the batch.
#ifndef MR_WAVES_PER_SIMD
#define MR_WAVES_PER_SIMD 2
#endif
template <typename T, int MODEL>
__global__ __launch_bounds__(WL, MR_WAVES_PER_SIMD) void mr_wave_kernel(ProbParams<T> P, mr_inputs in, mr_outputs out, int B, T* ws) {
  __shared__ T lds[LDS_WORDS];
  const int i = blockIdx.x;
  Wv w{(int)threadIdx.x};
  solve_instance_wave<T, MODEL>(P, in, out, B, i, (MR_GLOBAL T*)(ws + (int64_t)i * WS_WORDS), (MR_LDS T*)lds, w);
}

static size_t ws_bytes_per_instance(const mr_config& c) {
  return (size_t)WS_WORDS * (c.precision == MR_PREC_FP32 ? sizeof(float) : sizeof(double));
}

template <typename T, int MODEL>
static int launch(mr_handle* h, int B, const mr_inputs* in, mr_outputs* out, hipStream_t st) {
  ProbParams<T> P;
  fill_params<T>(h->cfg, h->tf, h->tr, P);
  hipLaunchKernelGGL((mr_wave_kernel<T, MODEL>), dim3(B), dim3(WL), 0, st, P, *in, *out, B, (T*)h->ws);
  HIP_TRY(hipGetLastError());
  return MR_OK;
}

template <typename T>
static int dispatch_model(mr_handle* h, int B, const mr_inputs* in, mr_outputs* out, hipStream_t st) {
  switch (h->cfg.model) {
    case MR_MODEL_KINEMATIC: return launch<T, MODEL_KIN>(h, B, in, out, st);
    case MR_MODEL_DYNAMIC: return launch<T, MODEL_DYN>(h, B, in, out, st);
    case MR_MODEL_BLENDED: return launch<T, MODEL_BLEND>(h, B, in, out, st);
    case MR_MODEL_BLENDED_PACEJKA: return launch<T, MODEL_BLEND_PACEJKA>(h, B, in, out, st);
    case MR_MODEL_DYNAMIC_PACEJKA: return launch<T, MODEL_DYN_PACEJKA>(h, B, in, out, st);
  }
  return fail(MR_ERR_ARG, "unknown model");
}

template <int MODEL>
__global__ void mr_eval_dynamics_kernel(ProbParams<double> P, int n, const double* x, const double* u,
                                        const double* nu, double* f, double* J, double* H) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (J == nullptr)  // value-only variant (used by the rollout / line search)
    Dyn<double, MODEL>::f(P, x + 6 * i, u + 2 * i, f + 6 * i);
  else
    Dyn<double, MODEL>::fjh(P, x + 6 * i, u + 2 * i, nu + 6 * i, f + 6 * i, J + 48 * i, H + 36 * i);
}

extern "C" {

int mr_version(void) { return 100; }

int mr_eval_dynamics(mr_handle* h, int32_t n, const double* x, const double* u, const double* nu, double* f,
                     double* J, double* H, void* hip_stream) {
  if (!h || !x || !u || !f || n < 0 || (J && (!H || !nu))) return fail(MR_ERR_ARG, "null argument");
  ProbParams<double> P;
  fill_params<double>(h->cfg, h->tf, h->tr, P);
  hipStream_t st = (hipStream_t)hip_stream;
  dim3 grid((n + 63) / 64), block(64);
  switch (h->cfg.model) {
    case MR_MODEL_KINEMATIC: hipLaunchKernelGGL(mr_eval_dynamics_kernel<MODEL_KIN>, grid, block, 0, st, P, n, x, u, nu, f, J, H); break;
    case MR_MODEL_DYNAMIC: hipLaunchKernelGGL(mr_eval_dynamics_kernel<MODEL_DYN>, grid, block, 0, st, P, n, x, u, nu, f, J, H); break;
    case MR_MODEL_BLENDED: hipLaunchKernelGGL(mr_eval_dynamics_kernel<MODEL_BLEND>, grid, block, 0, st, P, n, x, u, nu, f, J, H); break;
    case MR_MODEL_BLENDED_PACEJKA: hipLaunchKernelGGL(mr_eval_dynamics_kernel<MODEL_BLEND_PACEJKA>, grid, block, 0, st, P, n, x, u, nu, f, J, H); break;
    case MR_MODEL_DYNAMIC_PACEJKA: hipLaunchKernelGGL(mr_eval_dynamics_kernel<MODEL_DYN_PACEJKA>, grid, block, 0, st, P, n, x, u, nu, f, J, H); break;
    default: return fail(MR_ERR_ARG, "unknown model");
  }
  HIP_TRY(hipGetLastError());
  return MR_OK;
}

const char* mr_last_error(void) { return g_err.c_str(); }

int mr_config_default(mr_config* cfg) {
  if (!cfg) return fail(MR_ERR_ARG, "null config");
  fill_default_config(cfg);
  return MR_OK;
}

int mr_create(mr_handle** out, const mr_config* cfg) {
  if (!out || !cfg) return fail(MR_ERR_ARG, "null argument");
  if (cfg->N < 1 || cfg->N > WL - 1) return fail(MR_ERR_ARG, "N out of range (1..63: one wavefront lane per stage)");
  if (cfg->model < 0 || cfg->model > 4) return fail(MR_ERR_ARG, "unknown model");
  if (cfg->precision != MR_PREC_FP64 && cfg->precision != MR_PREC_FP32) return fail(MR_ERR_ARG, "bad precision");
  if (cfg->max_batch < 1) return fail(MR_ERR_ARG, "max_batch < 1");
  if (!(cfg->Ts > 0)) return fail(MR_ERR_ARG, "Ts must be > 0");
  HIP_TRY(hipSetDevice(cfg->device));
  mr_handle* h = new mr_handle();
  h->cfg = *cfg;
  h->have_tyres = 0;
  memset(&h->tf, 0, sizeof(h->tf));
  memset(&h->tr, 0, sizeof(h->tr));
  h->ws_bytes = ws_bytes_per_instance(*cfg) * (size_t)cfg->max_batch;
  hipError_t e = hipMalloc(&h->ws, h->ws_bytes);
  if (e != hipSuccess) {
    delete h;
    return fail(MR_ERR_HIP, std::string("workspace hipMalloc: ") + hipGetErrorString(e));
  }
  *out = h;
  return MR_OK;
}

int mr_destroy(mr_handle* h) {
  if (!h) return MR_OK;
  if (h->ws) (void)hipFree(h->ws);
  delete h;
  return MR_OK;
}

int mr_set_tyres(mr_handle* h, const double* a_front, double Fz_front, const double* a_back, double Fz_back) {
  if (!h || !a_front || !a_back) return fail(MR_ERR_ARG, "null argument");
  h->tf = pacejka_coef(a_front, Fz_front);
  h->tr = pacejka_coef(a_back, Fz_back);
  h->have_tyres = 1;
  return MR_OK;
}

int64_t mr_workspace_bytes_per_instance(const mr_handle* h) {
  return h ? (int64_t)ws_bytes_per_instance(h->cfg) : -1;
}

int mr_solve_batch(mr_handle* h, int32_t B, const mr_inputs* in, mr_outputs* out, void* hip_stream) {
  if (!h || !in || !out) return fail(MR_ERR_ARG, "null argument");
  if (B < 0 || B > h->cfg.max_batch) return fail(MR_ERR_ARG, "B exceeds max_batch");
  if (B == 0) return MR_OK;
  if (!in->state0 || !in->s0 || !in->cx || !in->cy || !in->max_error || !in->runtime)
    return fail(MR_ERR_ARG, "missing input array");
  if (!out->X || !out->U || !out->S || !out->eC || !out->eL || !out->status || !out->iters)
    return fail(MR_ERR_ARG, "missing output array");
  const int m = h->cfg.model;
  if ((m == MR_MODEL_BLENDED_PACEJKA || m == MR_MODEL_DYNAMIC_PACEJKA) && !h->have_tyres)
    return fail(MR_ERR_STATE, "Pacejka model needs mr_set_tyres");
  HIP_TRY(hipSetDevice(h->cfg.device));
  hipStream_t st = (hipStream_t)hip_stream;
  if (h->cfg.precision == MR_PREC_FP64) return dispatch_model<double>(h, B, in, out, st);
  return dispatch_model<float>(h, B, in, out, st);
}

}  // extern "C"
