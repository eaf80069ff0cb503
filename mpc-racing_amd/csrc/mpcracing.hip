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
// The centerline, sensing and plant kernels are bit-exact against the host build and the oracle
// (tests/test_gpu_track.py, test_lane_table.py, test_gpu_closed_loop.py): no FMA contraction in the
// code below (the solver above is built with -ffp-contract=fast, build.py).
#pragma clang fp contract(off)
#include "mr_track.h"
#include "mr_agent.h"
#include "mr_plant.h"
#include <vector>

using namespace mr;

struct mr_handle {
  mr_config cfg;
  void* params_dev;  // ProbParams<T> of the handle's precision (device copy, set by upload_params)
  void* ws;
  size_t ws_bytes;
  int* order;  // [2][max_batch] workgroup -> instance (mr_order_kernel), then mr_order_hint_kernel's buckets
  int32_t* last_iters;  // [max_batch] the previous solve's iterations (dispatch_order 2's default hint)
  int last_B;           // batch size of that solve (0: none yet)
  TyreCoef<double> tf, tr;
  int have_tyres;
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// Entry points switch to the handle's device for their HIP calls and restore the caller's current
// device on return (a library call must not change it).  A device that cannot be made current is an
// error of the entry point (MR_GUARD_DEVICE), never a silent launch on whatever device is current.
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};
#define MR_GUARD_DEVICE(dev)                                                                       \
  DeviceGuard dg_(dev);                                                                            \
  if (dg_.err != hipSuccess)                                                                       \
    return fail(MR_ERR_HIP, std::string("hipSetDevice(") + std::to_string(dev) + "): " + hipGetErrorString(dg_.err))

// The device that owns a device pointer (entry points without a handle: mr_plant_step).
static int pointer_device(const void* p, int* dev) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) return -1;
  if (a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged) return -1;
  *dev = a.device;
  return 0;
}

#define HIP_TRY(x)                                                                  \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) return fail(MR_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// One 64-lane workgroup (= one wavefront) per instance: lanes are stages / matrix rows
// of that instance (mr_wave.h); the grid is the batch.
// Waves per SIMD (launch bounds): fp32 2 -- the sweeps fit 256 registers with few spills (the
// generated dynamics code built without SLP vectorisation, build.py), and a second resident wave
// hides part of each instance's serial latency (A/B: profiles/r03_flags_ab.json, tools/gpu_flags_ab.sh);
// fp64 1 -- its sweeps need the full 512-register file (C3 0.418 vs 0.389 s at 2 vs 1 in round 1).
#ifndef MR_WAVES_PER_SIMD_F32
#define MR_WAVES_PER_SIMD_F32 2
#endif
#ifndef MR_WAVES_PER_SIMD_F64
#define MR_WAVES_PER_SIMD_F64 1
#endif
// Option (MR_SS_LDS=1, fp32 only): the per-stage fields (ss, 38.9 KB) live in LDS, so the
// sweeps' field loads are LDS round trips instead of Infinity-Cache / HBM ones.  Measured on C4:
// same iterates, B = 1 latency 5.31 -> 4.98 ms, but 44.4 KB of LDS per workgroup leaves 3
// instances per CU instead of 4 and the 8 192-instance batch takes 107.6 ms instead of 103.5 ms.
// Off by default.
#ifndef MR_SS_LDS
#define MR_SS_LDS 0
#endif
template <typename T>
struct SSInLDS { static constexpr bool value = MR_SS_LDS && sizeof(T) == 4; };

template <typename T, int MODEL>
__global__ __launch_bounds__(WL, sizeof(T) == 4 ? MR_WAVES_PER_SIMD_F32 : MR_WAVES_PER_SIMD_F64) void mr_wave_kernel(const ProbParams<T>* Pdev, mr_inputs in, mr_outputs out, int B,
                                                                         T* ws, const int* order) {
  __shared__ alignas(16) T lds[LDS_WORDS];
  const int i = order ? order[blockIdx.x] : (int)blockIdx.x;
  const int64_t t_start = out.timeline ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  Wv w{(int)threadIdx.x};
  MR_GLOBAL T* wsi = (MR_GLOBAL T*)(ws + (int64_t)i * ws_words<T>());
  // problem constants: the handle's device copy, read through the constant address space (scalar
  // loads, SGPRs); instance constants in LDS (every lane writes the same values)
  const MR_CONST ProbParams<T>& P = *(const MR_CONST ProbParams<T>*)Pdev;
  __shared__ Inst<T> Ish;
  // one solver object per lane (its wave-uniform iteration state), also in LDS
  constexpr bool SSL = SSInLDS<T>::value;
  __shared__ alignas(16) char slots[WL * sizeof(WaveSolver<T, MODEL, SSL>)];
  __shared__ WaveShared<T> wsh;  // the line-search filter and the watchdog / restoration state, shared by the wave
  T* const filt_sh = wsh.filt;
#ifdef MR_POISON
  {  // developer check (tools/determinism_probe.py): LDS and the instance's workspace start as a fixed pattern,
     // 1 NaN / 2 zero / 3 -1e30, so a read before the solve's first write shows as a difference between patterns
    const T pv = MR_POISON == 1 ? (T)NAN : MR_POISON == 2 ? T(0) : T(-1e30);
    for (int q = threadIdx.x; q < LDS_WORDS; q += WL) lds[q] = pv;
    for (int q = threadIdx.x; q < (int)(sizeof(slots) / sizeof(T)); q += WL) ((T*)slots)[q] = pv;
    for (int q = threadIdx.x; q < (int)(sizeof(wsh) / sizeof(T)); q += WL) ((T*)&wsh)[q] = pv;
    for (int q = threadIdx.x; q < (int)(sizeof(Ish) / sizeof(T)); q += WL) ((T*)&Ish)[q] = pv;
    for (int64_t q = threadIdx.x; q < ws_words<T>(); q += WL) wsi[q] = pv;
    __syncthreads();
  }
#endif
  if constexpr (SSL) {
    __shared__ T ssl[SS_WORDS];
    solve_instance_wave<T, MODEL, true, true>(P, in, out, B, i, wsi, (MR_LDS T*)lds, w, (MR_LDS T*)ssl, &Ish,
                                              slots, (MR_LDS T*)filt_sh);
  } else {
    solve_instance_wave<T, MODEL, false, true>(P, in, out, B, i, wsi, (MR_LDS T*)lds, w, wsi, &Ish, slots,
                                               (MR_LDS T*)filt_sh);
  }
  if (out.timeline && threadIdx.x == 0) {
    out.timeline[i] = t_start;
    out.timeline[(int64_t)B + i] = (int64_t)__builtin_amdgcn_s_memrealtime();
  }
}

// Dispatch order (mr_config.dispatch_order = 1): a stable three-tier partition of the batch so that
// the solves likely to run hundreds of iterations start first -- workgroups are dispatched roughly
// in index order, and a long solve that starts late extends the batch (profiles/r02_C4_timeline_*).
//   tier 0: near the top speed (v >= 40 m/s), or under hard braking (throttle0 <= -0.5) at v <= 20 m/s:
//           with the throttle rate limit the predicted car decelerates through a blend corner of the
//           model (Vblendmax = 15 m/s, Vblendmin = 2 m/s, models/VehicleParameters.py:37-38) within the
//           horizon -- 23 % of C4 (fits the first dispatch round), 26 of its 30 solves >= 300 iterations;
//   tier 1: the other instances outside 16.5 < v < 39 (the Vblendmax = 15 m/s blend corner nearby,
//           or fast);
//   tier 2: the rest.
// One workgroup of 1024 threads: per-thread chunk counts per tier, two LDS scans, then every thread
// writes its chunk.  NaN speeds go to tier 0.
constexpr int kOrderThreads = 1024;
__device__ __forceinline__ int order_tier(const double* state0, int B, int i) {
  const double vx = state0[3 * (int64_t)B + i], vy = state0[4 * (int64_t)B + i], thr = state0[6 * (int64_t)B + i];
  const double v = sqrt(vx * vx + vy * vy);
  if (!(v < 40.0) || (v <= 20.0 && thr <= -0.5)) return 0;
  return (v > 16.5 && v < 39.0) ? 2 : 1;
}
__device__ __forceinline__ int order_scan(int* cnt, int t, int c) {  // inclusive scan of c over the block
  cnt[t] = c;
  __syncthreads();
  for (int off = 1; off < kOrderThreads; off <<= 1) {  // Hillis-Steele
    const int v = t >= off ? cnt[t - off] : 0;
    __syncthreads();
    cnt[t] += v;
    __syncthreads();
  }
  const int r = cnt[t];
  __syncthreads();
  return r;
}
__device__ void order_tiers(const double* state0, int B, int* order, int* cnt, int* tot) {
  const int t = threadIdx.x;
  const int per = (B + kOrderThreads - 1) / kOrderThreads;
  const int lo = min(B, t * per), hi = min(B, lo + per);
  int c0 = 0, c1 = 0;
  for (int i = lo; i < hi; ++i) {
    const int q = order_tier(state0, B, i);
    c0 += q == 0;
    c1 += q == 1;
  }
  const int s0 = order_scan(cnt, t, c0);
  if (t == kOrderThreads - 1) tot[0] = s0;
  const int s1 = order_scan(cnt, t, c1);
  if (t == kOrderThreads - 1) tot[1] = s1;
  __syncthreads();
  int p0 = s0 - c0;                          // tier-0 slots before this chunk
  int p1 = tot[0] + (s1 - c1);               // tier 1 after all of tier 0
  int p2 = tot[0] + tot[1] + (lo - (s0 - c0) - (s1 - c1));  // tier 2 after both
  for (int i = lo; i < hi; ++i) {
    const int q = order_tier(state0, B, i);
    if (q == 0) order[p0++] = i;
    else if (q == 1) order[p1++] = i;
    else order[p2++] = i;
  }
}
__global__ __launch_bounds__(kOrderThreads) void mr_order_kernel(const double* state0, int B, int* order) {
  __shared__ int cnt[kOrderThreads];
  __shared__ int tot[2];
  order_tiers(state0, B, order, cnt, tot);
}

// dispatch_order = 2: workgroups take instances in decreasing order_hint (longest expected first), e.g.
// the previous MPC tick's iteration counts.  One workgroup: each hint is read ONCE into a bucket index
// (clamped to 0..kHintBuckets-1, kept in `bucket`, the second half of the handle's order buffer), a bucket
// histogram in LDS, a scan from the largest bucket down, then an atomic scatter from the stored buckets (the
// order within a bucket is arbitrary; results do not depend on the order).  Reading the hint once keeps
// `order` a permutation even if the hint buffer changes under the kernel (a caller's unordered stream); the
// scatter index is clamped to the batch besides.  A hint that says nothing (every instance in one bucket,
// e.g. all zero) gives instance order: no model-specific guess.
constexpr int kHintBuckets = kOrderThreads;
__device__ __forceinline__ int hint_bucket(int h) { return h < 0 ? 0 : (h >= kHintBuckets ? kHintBuckets - 1 : h); }
__global__ __launch_bounds__(kOrderThreads) void mr_order_hint_kernel(const int32_t* hint, int B, int* order,
                                                                       int* bucket) {
  __shared__ int cnt[kHintBuckets];
  __shared__ int scan[kOrderThreads];
  __shared__ int b0;
  const int t = threadIdx.x;
  cnt[t] = 0;
  __syncthreads();
  for (int i = t; i < B; i += kOrderThreads) {
    const int b = hint_bucket(hint[i]);
    bucket[i] = b;
    if (i == 0) b0 = b;
    atomicAdd(&cnt[b], 1);
  }
  __syncthreads();
  if (cnt[b0] == B) {  // uniform hint (block-uniform branch): instance order
    for (int i = t; i < B; i += kOrderThreads) order[i] = i;
    return;
  }
  const int r = kHintBuckets - 1 - t;  // thread t scans bucket r: the largest bucket first
  const int c = cnt[r];
  const int incl = order_scan(scan, t, c);
  cnt[r] = incl - c;  // first slot of bucket r
  __syncthreads();
  for (int i = t; i < B; i += kOrderThreads) {
    const int slot = atomicAdd(&cnt[bucket[i]], 1);  // this thread's own bucket store: no fence needed
    if (slot < B) order[slot] = i;
  }
}

static size_t ws_bytes_per_instance(const mr_config& c) {
  return c.precision == MR_PREC_FP32 ? (size_t)ws_words<float>() * sizeof(float) : (size_t)ws_words<double>() * sizeof(double);
}

// The handle's problem constants to its device buffer (mr_create, mr_set_tyres): the kernels read them
// through the constant address space.
static int upload_params(mr_handle* h) {
  if (h->cfg.precision == MR_PREC_FP64) {
    ProbParams<double> P;
    fill_params<double>(h->cfg, h->tf, h->tr, P);
    HIP_TRY(hipMemcpy(h->params_dev, &P, sizeof(P), hipMemcpyHostToDevice));
  } else {
    ProbParams<float> P;
    fill_params<float>(h->cfg, h->tf, h->tr, P);
    HIP_TRY(hipMemcpy(h->params_dev, &P, sizeof(P), hipMemcpyHostToDevice));
  }
  return MR_OK;
}

template <typename T, int MODEL>
static int launch(mr_handle* h, int B, const mr_inputs* in, mr_outputs* out, hipStream_t st) {
  const int* order = nullptr;
  if (h->cfg.dispatch_order == 1 && B > 1) {
    hipLaunchKernelGGL(mr_order_kernel, dim3(1), dim3(kOrderThreads), 0, st, in->state0, B, h->order);
    HIP_TRY(hipGetLastError());
    order = h->order;
  } else if (h->cfg.dispatch_order == 2 && B > 1) {
    // the caller's hint, else the handle's previous solve of the same batch size (the closed loop's
    // previous tick), else instance order -- no model-specific guess
    const int32_t* hint = in->order_hint ? in->order_hint : (h->last_B == B ? h->last_iters : nullptr);
    if (hint) {
      hipLaunchKernelGGL(mr_order_hint_kernel, dim3(1), dim3(kOrderThreads), 0, st, hint, B, h->order,
                         h->order + h->cfg.max_batch);
      HIP_TRY(hipGetLastError());
      order = h->order;
    }
  }
  hipLaunchKernelGGL((mr_wave_kernel<T, MODEL>), dim3(B), dim3(WL), 0, st, (const ProbParams<T>*)h->params_dev, *in,
                     *out, B, (T*)h->ws, order);
  HIP_TRY(hipGetLastError());
  if (h->cfg.dispatch_order == 2) {  // this solve's iterations: the next call's default hint
    HIP_TRY(hipMemcpyAsync(h->last_iters, out->iters, sizeof(int32_t) * (size_t)B, hipMemcpyDeviceToDevice, st));
    h->last_B = B;
  }
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


// ---------------------------------------------------------------------------------------------
// Centerline geometry kernels (mr_track.h): one lane per query, 256-lane workgroups.
// ---------------------------------------------------------------------------------------------
struct mr_track {
  int device;
  int nt, n_rows;
  double L;
  double* blob;  // device tables (track_layout)
  TrackView view;
};

constexpr int kTrackBlock = 256;

__global__ __launch_bounds__(kTrackBlock) void mr_track_eval_kernel(TrackView T, int n, const double* s, double* out,
                                                                    int32_t* span) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  double g[6];
  int sp;
  track_eval(T, s[i], g, &sp);
  for (int c = 0; c < 6; ++c) out[(int64_t)c * n + i] = g[c];
  if (span) span[i] = sp;
}

__global__ __launch_bounds__(kTrackBlock) void mr_track_frame_kernel(TrackView T, int n, const double* s, double* yaw,
                                                                     double* kappa, double* nx, double* ny, double mcla,
                                                                     double* meank) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  double y, k, a, b;
  track_frame(T, s[i], &y, &k, &a, &b);
  if (yaw) yaw[i] = y;
  if (kappa) kappa[i] = k;
  if (nx) nx[i] = a;
  if (ny) ny[i] = b;
  if (meank) meank[i] = track_mean_curvature(T, s[i], mcla);
}

__global__ __launch_bounds__(kTrackBlock) void mr_track_sign_kernel(TrackView T, int n, const double* X, const double* Y,
                                                                    const double* s, int32_t* sign) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  sign[i] = track_error_sign(T, X[i], Y[i], s[i]);
}

__global__ __launch_bounds__(kTrackBlock) void mr_track_polyfit_kernel(TrackView T, int n, const double* s,
                                                                       const double* la, double* cx, double* cy) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  double a[5], b[5];
  track_polyfit(T, s[i], la[i], a, b);
  for (int j = 0; j < 5; ++j) { cx[(int64_t)j * n + i] = a[j]; cy[(int64_t)j * n + i] = b[j]; }
}

__global__ __launch_bounds__(kTrackBlock) void mr_track_polyfit_deg_kernel(TrackView T, int n, const double* s,
                                                                           const double* la, int deg, double* cx,
                                                                           double* cy) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  double a[MR_POLY_DEG_MAX + 1], b[MR_POLY_DEG_MAX + 1];
  if (!track_polyfit_deg(T, s[i], la[i], deg, a, b)) return;
  for (int j = 0; j <= deg; ++j) { cx[(int64_t)j * n + i] = a[j]; cy[(int64_t)j * n + i] = b[j]; }
}

__global__ __launch_bounds__(kTrackBlock) void mr_track_lookup_kernel(TrackView T, int n, const double* s,
                                                                      const double* la, double* err, int32_t* rlo,
                                                                      int32_t* rhi, int32_t* rarg) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  int lo, hi, arg;
  err[i] = lane_lookup(T, s[i], la[i], &lo, &hi, &arg);
  if (rlo) rlo[i] = lo;
  if (rhi) rhi[i] = hi;
  if (rarg) rarg[i] = arg;
}

__global__ __launch_bounds__(kTrackBlock) void mr_track_projection_kernel(TrackView T, int n, const double* X,
                                                                          const double* Y, const double* lo,
                                                                          const double* hi, double* s, double* dist,
                                                                          int32_t* nfev) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  int nf;
  const double x = brent_projection(T, X[i], Y[i], lo[i], hi[i], &nf);
  s[i] = x;
  dist[i] = track_dist(T, x, X[i], Y[i]);
  if (nfev) nfev[i] = nf;
}

__global__ __launch_bounds__(kTrackBlock) void mr_track_prep_kernel(TrackView T, int n, const double* X, const double* Y,
                                                                    const double* lo, const double* hi, double lookback,
                                                                    double lookahead, double err_offset, double* s,
                                                                    double* dist, double* cx, double* cy, double* merr) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  const double p = brent_projection(T, X[i], Y[i], lo[i], hi[i], nullptr);
  s[i] = p;
  dist[i] = track_dist(T, p, X[i], Y[i]);
  double a[5], b[5];
  track_polyfit(T, p - lookback, lookahead, a, b);
  for (int j = 0; j < 5; ++j) { cx[(int64_t)j * n + i] = a[j]; cy[(int64_t)j * n + i] = b[j]; }
  merr[i] = lane_lookup(T, p, lookahead, nullptr, nullptr, nullptr) - err_offset;
}

// Closed-loop pieces (mr_agent.h, mr_plant.h): one lane per vehicle.
// Lane-width table build (mr_track.h lane_distance): one wavefront per centerline sample.
// Lane l scans lane-spline samples m = l, l + 64, ... (knot-interval start / midpoint, span
// known, no search); the wave arg-min (smallest m on ties, as the serial scan) brackets the
// bounded-Brent refinement, which lane 0 runs.  The lane tables (~0.5 MB for Shanghai) stay
// L2-resident across the grid.
constexpr int kLaneWaves = 4;
__global__ __launch_bounds__(64 * kLaneWaves) void mr_lane_table_kernel(TrackView C, TrackView lane, int n,
                                                                       const double* s, double* dist,
                                                                       double* s_lane) {
  const int q = blockIdx.x * kLaneWaves + (int)(threadIdx.x >> 6);
  const int ln = (int)(threadIdx.x & 63);
  if (q >= n) return;  // wave-uniform
  double X, Y;
  centerline_point(C, s[q], &X, &Y);
  const int M = lane_n_samples(lane);
  double best = 1e300;
  int mb = 0x7fffffff;
  for (int m = ln; m < M; m += 64) {
    const double d2 = lane_sample_d2(lane, m, X, Y);
    if (d2 < best) { best = d2; mb = m; }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    const double od = __shfl_xor(best, off);
    const int om = __shfl_xor(mb, off);
    if (od < best || (od == best && om < mb)) { best = od; mb = om; }
  }
  if (ln == 0) {
    double u;
    dist[q] = lane_refine(lane, X, Y, mb, &u);
    if (s_lane) s_lane[q] = u;
  }
}

__global__ __launch_bounds__(kTrackBlock) void mr_agent_sense_kernel(TrackView T, int n, const double* X, const double* Y,
                                                                     const double* prev, double lookback, double lookahead,
                                                                     double err_offset, double* progress, double* error,
                                                                     double* cx, double* cy, double* merr) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  AgentSense o;
  agent_sense(T, X[i], Y[i], prev ? prev[i] : NAN, lookback, lookahead, err_offset, o);
  progress[i] = o.progress;
  error[i] = o.error;
  for (int j = 0; j < 5; ++j) { cx[(int64_t)j * n + i] = o.cx[j]; cy[(int64_t)j * n + i] = o.cy[j]; }
  merr[i] = o.max_error;
}

__global__ __launch_bounds__(kTrackBlock) void mr_plant_step_kernel(int model, int n, const double* state,
                                                                    const double* cmd, double dt, double* out) {
  const int i = blockIdx.x * kTrackBlock + threadIdx.x;
  if (i >= n) return;
  double x[6], o[6];
  for (int j = 0; j < 6; ++j) x[j] = state[(int64_t)j * n + i];
  plant_step(model, x, cmd[i], cmd[n + i], dt, o);
  for (int j = 0; j < 6; ++j) out[(int64_t)j * n + i] = o[j];
}

extern "C" {

int mr_version(void) { return MR_ABI_VERSION; }

int mr_eval_dynamics(mr_handle* h, int32_t n, const double* x, const double* u, const double* nu, double* f,
                     double* J, double* H, void* hip_stream) {
  if (!h || !x || !u || !f || n < 0 || (J && (!H || !nu))) return fail(MR_ERR_ARG, "null argument");
  MR_GUARD_DEVICE(h->cfg.device);
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
  // the line-search filter holds FCAP entries (mr_solver.h): at most one per iteration plus the restoration
  // entry's, so a solve with max_iter <= FCAP - 2 never drops one (IPOPT's filter is unbounded)
  if (cfg->max_iter < 0 || cfg->max_iter > FCAP - 2)
    return fail(MR_ERR_ARG, "max_iter out of range (0.." + std::to_string(FCAP - 2) + ": the line-search filter's capacity)");
  if (!(cfg->Ts > 0)) return fail(MR_ERR_ARG, "Ts must be > 0");
  if (cfg->dispatch_order < 0 || cfg->dispatch_order > 2) return fail(MR_ERR_ARG, "dispatch_order must be 0, 1 or 2");
  {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    if (cfg->device < 0 || cfg->device >= ndev)
      return fail(MR_ERR_ARG, "device " + std::to_string(cfg->device) + " out of range (" + std::to_string(ndev) +
                                  " HIP devices)");
  }
  MR_GUARD_DEVICE(cfg->device);
  mr_handle* h = new mr_handle();
  h->cfg = *cfg;
  h->have_tyres = 0;
  memset(&h->tf, 0, sizeof(h->tf));
  memset(&h->tr, 0, sizeof(h->tr));
  h->ws_bytes = ws_bytes_per_instance(*cfg) * (size_t)cfg->max_batch;
  h->order = nullptr;
  h->last_iters = nullptr;
  h->last_B = 0;
  hipError_t e = hipMalloc(&h->ws, h->ws_bytes);
  if (e == hipSuccess) e = hipMalloc((void**)&h->order, 2 * sizeof(int) * (size_t)cfg->max_batch);  // + the hint buckets
  if (e == hipSuccess) e = hipMalloc((void**)&h->last_iters, sizeof(int32_t) * (size_t)cfg->max_batch);
  if (e == hipSuccess) e = hipMalloc(&h->params_dev, sizeof(ProbParams<double>));
  if (e != hipSuccess) {
    if (h->ws) (void)hipFree(h->ws);
    if (h->order) (void)hipFree(h->order);
    if (h->last_iters) (void)hipFree(h->last_iters);
    delete h;
    return fail(MR_ERR_HIP, std::string("workspace hipMalloc: ") + hipGetErrorString(e));
  }
  {
    const int rc = upload_params(h);
    if (rc != MR_OK) {
      mr_destroy(h);
      return rc;
    }
  }
  *out = h;
  return MR_OK;
}

int mr_destroy(mr_handle* h) {
  if (!h) return MR_OK;
  if (h->ws) (void)hipFree(h->ws);
  if (h->order) (void)hipFree(h->order);
  if (h->last_iters) (void)hipFree(h->last_iters);
  if (h->params_dev) (void)hipFree(h->params_dev);
  delete h;
  return MR_OK;
}

int mr_set_tyres(mr_handle* h, const double* a_front, double Fz_front, const double* a_back, double Fz_back) {
  if (!h || !a_front || !a_back) return fail(MR_ERR_ARG, "null argument");
  MR_GUARD_DEVICE(h->cfg.device);
  // the kernels read the constants from this buffer while they run: a solve still in flight on any
  // stream of the device (torch side streams do not order with the copy below) must finish first
  HIP_TRY(hipDeviceSynchronize());
  // the handle takes the new coefficients only once they are on the device
  const auto tf = h->tf, tr = h->tr;
  const int had = h->have_tyres;
  h->tf = pacejka_coef(a_front, Fz_front);
  h->tr = pacejka_coef(a_back, Fz_back);
  const int rc = upload_params(h);
  if (rc != MR_OK) {
    h->tf = tf;
    h->tr = tr;
    h->have_tyres = had;
    return rc;
  }
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
  MR_GUARD_DEVICE(h->cfg.device);
  hipStream_t st = (hipStream_t)hip_stream;
  if (h->cfg.precision == MR_PREC_FP64) return dispatch_model<double>(h, B, in, out, st);
  return dispatch_model<float>(h, B, in, out, st);
}


int mr_track_create(mr_track** out, int32_t device, const double* t, int32_t n_t, const double* cx, const double* cy,
                    int32_t n_c, double length, const double* err_left, const double* err_right, int32_t n_rows) {
  if (!out || !t || !cx || !cy) return fail(MR_ERR_ARG, "null argument");
  if (n_rows > 0 && (!err_left || !err_right)) return fail(MR_ERR_ARG, "null lane table");
  if (n_t < 8 || n_c < 4 || n_c > n_t || n_rows < 0 || !(length > 0)) return fail(MR_ERR_ARG, "bad track sizes");
  for (int i = 1; i < n_t; ++i)
    if (!(t[i] >= t[i - 1])) return fail(MR_ERR_ARG, "knots not sorted");
  const TrackLayout Lay = track_layout(n_t, n_rows);
  std::vector<double> blob(Lay.total);
  track_tables(t, n_t, cx, cy, n_c, err_left, err_right, n_rows, blob.data());
  {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    if (device < 0 || device >= ndev)
      return fail(MR_ERR_ARG, "device " + std::to_string(device) + " out of range (" + std::to_string(ndev) +
                                  " HIP devices)");
  }
  MR_GUARD_DEVICE(device);
  mr_track* tr = new mr_track();
  tr->device = device;
  tr->nt = n_t;
  tr->n_rows = n_rows;
  tr->L = length;
  hipError_t e = hipMalloc(&tr->blob, sizeof(double) * blob.size());
  if (e == hipSuccess) e = hipMemcpy(tr->blob, blob.data(), sizeof(double) * blob.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (tr->blob) (void)hipFree(tr->blob);
    delete tr;
    return fail(MR_ERR_HIP, std::string("track tables: ") + hipGetErrorString(e));
  }
  tr->view = track_view(tr->blob, n_t, length, n_rows);
  *out = tr;
  return MR_OK;
}

int mr_track_destroy(mr_track* tr) {
  if (!tr) return MR_OK;
  if (tr->blob) (void)hipFree(tr->blob);
  delete tr;
  return MR_OK;
}

#define MR_TRACK_LAUNCH(kernel, ...)                                                             \
  do {                                                                                           \
    if (!tr) return fail(MR_ERR_ARG, "null track");                                              \
    if (n < 0) return fail(MR_ERR_ARG, "n < 0");                                                 \
    if (n == 0) return MR_OK;                                                                    \
    MR_GUARD_DEVICE(tr->device);                                                                 \
    hipLaunchKernelGGL(kernel, dim3((n + kTrackBlock - 1) / kTrackBlock), dim3(kTrackBlock), 0,  \
                       (hipStream_t)hip_stream, tr->view, n, __VA_ARGS__);                       \
    HIP_TRY(hipGetLastError());                                                                  \
    return MR_OK;                                                                                \
  } while (0)

int mr_track_eval(const mr_track* tr, int32_t n, const double* s, double* out, int32_t* span, void* hip_stream) {
  if (!s || !out) return fail(MR_ERR_ARG, "null argument");
  MR_TRACK_LAUNCH(mr_track_eval_kernel, s, out, span);
}

int mr_track_frame(const mr_track* tr, int32_t n, const double* s, double* yaw, double* kappa, double* nx, double* ny,
                   double mc_lookahead, double* mean_kappa, void* hip_stream) {
  if (!s) return fail(MR_ERR_ARG, "null argument");
  MR_TRACK_LAUNCH(mr_track_frame_kernel, s, yaw, kappa, nx, ny, mc_lookahead, mean_kappa);
}

int mr_track_error_sign(const mr_track* tr, int32_t n, const double* X, const double* Y, const double* s,
                        int32_t* sign, void* hip_stream) {
  if (!X || !Y || !s || !sign) return fail(MR_ERR_ARG, "null argument");
  MR_TRACK_LAUNCH(mr_track_sign_kernel, X, Y, s, sign);
}

int mr_track_polyfit(const mr_track* tr, int32_t n, const double* s, const double* lookahead, double* cx, double* cy,
                     void* hip_stream) {
  if (!s || !lookahead || !cx || !cy) return fail(MR_ERR_ARG, "null argument");
  MR_TRACK_LAUNCH(mr_track_polyfit_kernel, s, lookahead, cx, cy);
}

int mr_track_polyfit_deg(const mr_track* tr, int32_t n, const double* s, const double* lookahead, int32_t deg,
                         double* cx, double* cy, void* hip_stream) {
  if (!s || !lookahead || !cx || !cy) return fail(MR_ERR_ARG, "null argument");
  if (deg < 0 || deg > MR_POLY_DEG_MAX) return fail(MR_ERR_ARG, "deg out of range (0..10)");
  MR_TRACK_LAUNCH(mr_track_polyfit_deg_kernel, s, lookahead, (int)deg, cx, cy);
}

int mr_track_lookup_error(const mr_track* tr, int32_t n, const double* s, const double* lookahead, double* err,
                          int32_t* row_lo, int32_t* row_hi, int32_t* row_arg, void* hip_stream) {
  if (!s || !lookahead || !err) return fail(MR_ERR_ARG, "null argument");
  MR_TRACK_LAUNCH(mr_track_lookup_kernel, s, lookahead, err, row_lo, row_hi, row_arg);
}

int mr_track_projection(const mr_track* tr, int32_t n, const double* X, const double* Y, const double* lo,
                        const double* hi, double* s, double* dist, int32_t* nfev, void* hip_stream) {
  if (!X || !Y || !lo || !hi || !s || !dist) return fail(MR_ERR_ARG, "null argument");
  MR_TRACK_LAUNCH(mr_track_projection_kernel, X, Y, lo, hi, s, dist, nfev);
}

int mr_track_prep(const mr_track* tr, int32_t n, const double* X, const double* Y, const double* lo, const double* hi,
                  double lookback, double lookahead, double err_offset, double* s, double* dist, double* cx,
                  double* cy, double* max_error, void* hip_stream) {
  if (!X || !Y || !lo || !hi || !s || !dist || !cx || !cy || !max_error) return fail(MR_ERR_ARG, "null argument");
  MR_TRACK_LAUNCH(mr_track_prep_kernel, X, Y, lo, hi, lookback, lookahead, err_offset, s, dist, cx, cy, max_error);
}

int mr_agent_sense(const mr_track* tr, int32_t n, const double* X, const double* Y, const double* prev_progress,
                   double lookback, double lookahead, double err_offset, double* progress, double* error, double* cx,
                   double* cy, double* max_error, void* hip_stream) {
  if (!X || !Y || !progress || !error || !cx || !cy || !max_error) return fail(MR_ERR_ARG, "null argument");
  MR_TRACK_LAUNCH(mr_agent_sense_kernel, X, Y, prev_progress, lookback, lookahead, err_offset, progress, error, cx, cy,
                  max_error);
}

int mr_spline_from_waypoints(const double* x, const double* y, int32_t n, int32_t close_loop, double* t, double* cx,
                             double* cy, int32_t* n_t, double* length) {
  if (!x || !y || !t || !cx || !cy || !n_t || !length) return fail(MR_ERR_ARG, "null argument");
  const int np = spline_from_waypoints(x, y, n, close_loop, t, cx, cy, length);
  if (np < 0) return fail(MR_ERR_ARG, "spline_from_waypoints: need >= 4 distinct waypoints in order");
  *n_t = np + 4;
  return MR_OK;
}

int mr_track_lane_table(const mr_track* centerline, const mr_track* lane, int32_t n, const double* s, double* dist,
                        double* s_lane, void* hip_stream) {
  if (!centerline || !lane || !s || !dist) return fail(MR_ERR_ARG, "null argument");
  if (centerline->device != lane->device) return fail(MR_ERR_ARG, "centerline and lane on different devices");
  if (n < 0) return fail(MR_ERR_ARG, "n < 0");
  if (n == 0) return MR_OK;
  MR_GUARD_DEVICE(centerline->device);
  hipLaunchKernelGGL(mr_lane_table_kernel, dim3((n + kLaneWaves - 1) / kLaneWaves), dim3(64 * kLaneWaves), 0,
                     (hipStream_t)hip_stream, centerline->view, lane->view, (int)n, s, dist, s_lane);
  HIP_TRY(hipGetLastError());
  return MR_OK;
}

int mr_plant_step(int32_t model, int32_t n, const double* state, const double* cmd, double dt, double* out,
                  void* hip_stream) {
  if (!state || !cmd || !out) return fail(MR_ERR_ARG, "null argument");
  if (model < MR_PLANT_KINEMATIC || model > MR_PLANT_BLENDED) return fail(MR_ERR_ARG, "unknown plant model");
  if (n < 0) return fail(MR_ERR_ARG, "n < 0");
  if (n == 0) return MR_OK;
  int dev = -1;
  if (pointer_device(state, &dev) != 0) return fail(MR_ERR_ARG, "state is not a HIP device pointer");
  MR_GUARD_DEVICE(dev);  // the arrays' device, not whichever device is current
  hipLaunchKernelGGL(mr_plant_step_kernel, dim3((n + kTrackBlock - 1) / kTrackBlock), dim3(kTrackBlock), 0,
                     (hipStream_t)hip_stream, (int)model, (int)n, state, cmd, dt, out);
  HIP_TRY(hipGetLastError());
  return MR_OK;
}

}  // extern "C"
