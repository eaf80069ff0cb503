// Wavefront primitives of the wave-per-instance solver (mr_wave.h).
//
// gfx950: one 64-lane wavefront = one workgroup = one MPC instance.  Cross-lane
// values move with ds_bpermute / v_readlane; LDS ordering inside the wave is a
// workgroup barrier (single-wave workgroup).
//
// Host (g++, TEST HARNESS ONLY): the same SPMD source runs as 64 cooperative
// fibers per instance (ucontext), every primitive a rendezvous of the 64 fibers,
// so the CPU test suite executes exactly the kernel's code path.  Reductions use
// the same butterfly order on both sides (bitwise-identical sums given identical
// inputs).  Every primitive must be reached by all 64 lanes (wave-uniform control
// flow), as on the device where an inactive source lane would read garbage.
#pragma once
#include "mr_common.h"

#if !MR_DEVICE_BUILD
#include <ucontext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <cmath>
#endif

// Address-space qualifiers: keep the workspace in the global and the exchange buffers in the
// LDS address space through the sweep functions (otherwise every access becomes a flat_* op
// that waits on both memory counters).
#if MR_DEVICE_BUILD
#define MR_GLOBAL __attribute__((address_space(1)))
#define MR_LDS __attribute__((address_space(3)))
#define MR_CONST __attribute__((address_space(4)))
#else
#define MR_GLOBAL
#define MR_LDS
#define MR_CONST
#endif

namespace mr {

constexpr int WL = 64;  // lanes per instance

#if MR_DEVICE_BUILD

struct Wv {
  int lane;
};

// Full sync: LDS and global memory written by any lane visible to every lane (workgroup
// release/acquire: waits for this wave's outstanding vector-memory operations).
__device__ __forceinline__ void wsync(const Wv&) { __syncthreads(); }
// LDS-only sync inside the single-wave workgroup: a wavefront's DS instructions execute in
// issue order, so a compiler-level barrier is enough; outstanding global loads (prefetches)
// and stores stay in flight.
__device__ __forceinline__ void wsync_lds(const Wv&) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float wshfl(const Wv&, float v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ double wshfl(const Wv&, double v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ int wshfl(const Wv&, int v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ float wxor(const Wv&, float v, int m) { return __shfl_xor(v, m, 64); }
__device__ __forceinline__ double wxor(const Wv&, double v, int m) { return __shfl_xor(v, m, 64); }
__device__ __forceinline__ int wxor(const Wv&, int v, int m) { return __shfl_xor(v, m, 64); }

// value of lane (lane + 1) mod 64 (the next stage's): one DPP row-crossing rotate (v_mov_b32_dpp wave_rol:1),
// a VALU move instead of a ds_bpermute through the CU's LDS crossbar
__device__ __forceinline__ float wnext(const Wv&, float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x134, 0xf, 0xf, false));
}
__device__ __forceinline__ double wnext(const Wv&, double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), 0x134, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x134, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// value of lane + 1 within the lane's row of 16 (0 for the row's last lane): v_mov_b32_dpp row_shl:1
__device__ __forceinline__ float wrow_next(const Wv&, float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xf, 0xf, true));
}
__device__ __forceinline__ double wrow_next(const Wv&, double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), 0x101, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x101, 0xf, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
// value of lane (lane - 1) mod 64 (the previous stage's): v_mov_b32_dpp wave_ror:1
__device__ __forceinline__ float wprev(const Wv&, float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x13C, 0xf, 0xf, false));
}
__device__ __forceinline__ double wprev(const Wv&, double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), 0x13C, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x13C, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// value of lane src (src wave-uniform): v_readlane, result lands in an SGPR
__device__ __forceinline__ int wbcast(const Wv&, int v, int src) { return __builtin_amdgcn_readlane(v, src); }
__device__ __forceinline__ float wbcast(const Wv&, float v, int src) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}
__device__ __forceinline__ double wbcast(const Wv&, double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// One 16x16x4 MFMA over the wave: D += A * B with lane l holding A[l&15][l>>4] and
// B[l>>4][l&15]; D row of register v: 4*(l>>4)+v (f32), (l>>4)+4*v (f64); column l&15.
typedef float mr_f32x4 __attribute__((ext_vector_type(4)));
typedef double mr_f64x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void wmfma(const Wv&, float a, float b, float* d) {
  mr_f32x4 c = {d[0], d[1], d[2], d[3]};
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  d[0] = c[0]; d[1] = c[1]; d[2] = c[2]; d[3] = c[3];
}
__device__ __forceinline__ void wmfma(const Wv&, double a, double b, double* d) {
  mr_f64x4 c = {d[0], d[1], d[2], d[3]};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  d[0] = c[0]; d[1] = c[1]; d[2] = c[2]; d[3] = c[3];
}

// A condition every lane computed identically, made visibly wave-uniform (SGPR) so branches
// on it stay scalar and the enclosing loop keeps a uniform counter and exact waitcnts.
__device__ __forceinline__ bool wuni(const Wv&, bool b) { return __builtin_amdgcn_readfirstlane((int)b) != 0; }
// any / every lane of the wave (one v_cmp into a lane mask; called in wave-uniform control flow)
__device__ __forceinline__ bool wany(const Wv&, bool b) { return __builtin_amdgcn_ballot_w64(b) != 0; }
__device__ __forceinline__ bool wall(const Wv&, bool b) { return __builtin_amdgcn_ballot_w64(!b) == 0; }
// A value every lane holds identically (e.g. reloaded from the per-lane solver object): SGPR copy
__device__ __forceinline__ int wu(const Wv&, int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float wu(const Wv&, float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ double wu(const Wv&, double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffLL));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// A pointer every lane holds identically, made visibly uniform (SGPR pair): loads through a
// constant-address-space pointer then become scalar loads (s_load into SGPRs) instead of per-lane
// vector loads into VGPRs -- the problem constants cost no vector registers.
template <typename T>
__device__ __forceinline__ const MR_CONST T* wu_ptr(const MR_CONST T* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (const MR_CONST T*)(((unsigned long long)hi << 32) | lo);
}

// the same for a global-memory base pointer (workspace of the instance): addresses become an SGPR
// base plus a 32-bit lane offset instead of per-lane 64-bit address arithmetic
template <typename T>
__device__ __forceinline__ MR_GLOBAL T* wu_gptr(MR_GLOBAL T* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (MR_GLOBAL T*)(((unsigned long long)hi << 32) | lo);
}

// the same for either address space: global pointers through readfirstlane, LDS ones unchanged
template <typename T>
__device__ __forceinline__ MR_GLOBAL T* wu_any(MR_GLOBAL T* p) { return wu_gptr(p); }
template <typename T>
__device__ __forceinline__ MR_LDS T* wu_any(MR_LDS T* p) { return p; }

// A wave-uniform global array addressed as (uniform word offset, per-lane word offset): a buffer
// resource in SGPRs, so every access is one buffer_load / buffer_store with a 32-bit lane offset
// VGPR and the uniform part in soffset -- no 64-bit per-lane address arithmetic, and no 64-bit
// address VGPR pair per gathered word held across a loop.
template <typename T>
struct WBuf {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ WBuf(MR_GLOBAL T* base, unsigned n_words)
      : r(__builtin_amdgcn_make_buffer_rsrc((void*)(T*)wu_gptr(base), 0, (int)(n_words * sizeof(T)), 0x00020000)) {}
  __device__ __forceinline__ T ld(unsigned uoff, unsigned loff) const {
    if constexpr (sizeof(T) == 4) {
      return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)(loff * 4u), (int)(uoff * 4u), 0));
    } else {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(loff * 8u), (int)(uoff * 8u), 0);
      return __longlong_as_double((long long)(((unsigned long long)v[1] << 32) | v[0]));
    }
  }
  __device__ __forceinline__ void st(T x, unsigned uoff, unsigned loff) const {
    if constexpr (sizeof(T) == 4) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, (int)(loff * 4u), (int)(uoff * 4u), 0);
    } else {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const unsigned long long b = (unsigned long long)__double_as_longlong(x);
      const u32x2 v = {(unsigned)b, (unsigned)(b >> 32)};
      __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)(loff * 8u), (int)(uoff * 8u), 0);
    }
  }
};

// out[i] = value of lane i, i < n (compile-time n): one v_readlane per element
template <typename T, int n>
__device__ __forceinline__ void wgather(const Wv& w, T v, T* out) {
#pragma unroll
  for (int i = 0; i < n; ++i) out[i] = wbcast(w, v, i);
}

// Wave reductions without LDS round trips: butterfly levels 1, 2 as DPP quad permutes, 4 and 8
// as DPP half-row / row mirrors (the same partners' values once quads / octets agree), 16 and
// 32 as the gfx950 v_permlane16_swap / v_permlane32_swap.  Every level computes
// op(own, partner) on every lane, as the xor butterfly does; the host emulation below uses the
// same partners in the same order, so sums round identically on both.
__device__ __forceinline__ int dpp_bits(int v, int ctrl_sel) {
  switch (ctrl_sel) {
    case 0: return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    case 1: return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    case 2: return __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, true);  // row_half_mirror
    default: return __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, true); // row_mirror
  }
}
__device__ __forceinline__ int bits_of(int v) { return v; }
__device__ __forceinline__ int bits_of(float v) { return __float_as_int(v); }
__device__ __forceinline__ void from_bits(int b, int& v) { v = b; }
__device__ __forceinline__ void from_bits(int b, float& v) { v = __int_as_float(b); }

template <typename T>
__device__ __forceinline__ T wdpp(T v, int sel) {
  if constexpr (sizeof(T) == 8) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_bits((int)(b & 0xffffffffLL), sel), hi = dpp_bits((int)(b >> 32), sel);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
  } else {
    T r;
    from_bits(dpp_bits(bits_of(v), sel), r);
    return r;
  }
}
// (own, partner) of butterfly level 16 (row pairs) or 32 (halves) on every lane
template <int LEVEL>
__device__ __forceinline__ void swap_bits(const Wv& w, int v, int& own, int& par) {
  const auto r = LEVEL == 16 ? __builtin_amdgcn_permlane16_swap(v, v, false, false)
                             : __builtin_amdgcn_permlane32_swap(v, v, false, false);
  const bool upper = LEVEL == 16 ? ((w.lane >> 4) & 1) : (w.lane >= 32);
  own = upper ? (int)r[1] : (int)r[0];
  par = upper ? (int)r[0] : (int)r[1];
}
template <int LEVEL, typename T>
__device__ __forceinline__ void wswap(const Wv& w, T v, T& own, T& par) {
  if constexpr (sizeof(T) == 8) {
    const long long b = __double_as_longlong(v);
    int ol, pl, oh, ph;
    swap_bits<LEVEL>(w, (int)(b & 0xffffffffLL), ol, pl);
    swap_bits<LEVEL>(w, (int)(b >> 32), oh, ph);
    own = __longlong_as_double(((long long)oh << 32) | (long long)(unsigned)ol);
    par = __longlong_as_double(((long long)ph << 32) | (long long)(unsigned)pl);
  } else {
    int o, q;
    swap_bits<LEVEL>(w, bits_of(v), o, q);
    from_bits(o, own);
    from_bits(q, par);
  }
}
template <typename T, typename Op>
__device__ __forceinline__ T wreduce(const Wv& w, T v, Op op) {
#pragma unroll
  for (int sel = 0; sel < 4; ++sel) v = op(v, wdpp(v, sel));
  T o, q;
  wswap<16>(w, v, o, q);
  v = op(o, q);
  wswap<32>(w, v, o, q);
  return op(o, q);
}
template <typename T>
__device__ __forceinline__ T wsum(const Wv& w, T v) {
  return wreduce(w, v, [](T a, T b) { return a + b; });
}
template <typename T>
__device__ __forceinline__ T wmax(const Wv& w, T v) {
  return wreduce(w, v, [](T a, T b) { return b > a ? b : a; });
}
template <typename T>
__device__ __forceinline__ T wmin(const Wv& w, T v) {
  return wreduce(w, v, [](T a, T b) { return b < a ? b : a; });
}

// 4x4 transpose across the four 16-lane rows of the wave, per column c = lane & 15: on entry lane
// (g, c) holds d[v] = M[g][v]; on exit d[s] = M[s][g].  This turns an f32 16x16x4 MFMA result
// (D layout: lane (g, c) register v = row 4g+v) into the next MFMA's B operand (register s = row
// 4s+g) without an LDS round trip: two v_permlane32_swap (rows {0,1} <-> {2,3}) and two
// v_permlane16_swap (rows 0 <-> 1, 2 <-> 3).
__device__ __forceinline__ void wtranspose4(const Wv&, float* d) {
  unsigned b0 = __float_as_uint(d[0]), b1 = __float_as_uint(d[1]), b2 = __float_as_uint(d[2]),
           b3 = __float_as_uint(d[3]);
  auto p02 = __builtin_amdgcn_permlane32_swap(b0, b2, false, false);
  auto p13 = __builtin_amdgcn_permlane32_swap(b1, b3, false, false);
  b0 = p02[0]; b2 = p02[1]; b1 = p13[0]; b3 = p13[1];
  auto p01 = __builtin_amdgcn_permlane16_swap(b0, b1, false, false);
  auto p23 = __builtin_amdgcn_permlane16_swap(b2, b3, false, false);
  d[0] = __uint_as_float(p01[0]); d[1] = __uint_as_float(p01[1]);
  d[2] = __uint_as_float(p23[0]); d[3] = __uint_as_float(p23[1]);
}

#else  // host fiber emulation -------------------------------------------------------------

struct HostWave {
  ucontext_t main_ctx;
  ucontext_t ctx[WL];
  char* stacks = nullptr;
  int cur = 0, arrived = 0, done = 0;
  int fin[WL];
  alignas(16) unsigned char buf[WL][16];
  void (*body)(HostWave*, int, void*) = nullptr;
  void* arg = nullptr;

  void barrier() {
    if (++arrived == WL) {
      arrived = 0;
      return;
    }
    const int me = cur;
    cur = (cur + 1) % WL;
    swapcontext(&ctx[me], &ctx[cur]);
  }
};

struct Wv {
  int lane;
  HostWave* hw;
};

inline void wsync(const Wv& w) { w.hw->barrier(); }
inline void wsync_lds(const Wv& w) { w.hw->barrier(); }

template <typename T>
inline T wshfl(const Wv& w, T v, int src) {
  memcpy(w.hw->buf[w.lane], &v, sizeof(T));
  w.hw->barrier();
  T r;
  memcpy(&r, w.hw->buf[((src % WL) + WL) % WL], sizeof(T));
  w.hw->barrier();
  return r;
}
template <typename T>
inline T wnext(const Wv& w, T v) { return wshfl(w, v, (w.lane + 1) % WL); }
template <typename T>
inline T wprev(const Wv& w, T v) { return wshfl(w, v, (w.lane + WL - 1) % WL); }
template <typename T>
inline T wrow_next(const Wv& w, T v) {
  const T r = wshfl(w, v, (w.lane & 15) < 15 ? w.lane + 1 : w.lane);
  return (w.lane & 15) < 15 ? r : T(0);
}
template <typename T>
inline T wbcast(const Wv& w, T v, int src) { return wshfl(w, v, src); }
template <typename T>
inline T wxor(const Wv& w, T v, int m) { return wshfl(w, v, w.lane ^ m); }

// 16x16x4 MFMA emulation: same lane maps and the same k-ordered fma chain as gfx950
template <typename T>
inline void wmfma(const Wv& w, T a, T b, T* d) {
  memcpy(w.hw->buf[w.lane], &a, sizeof(T));
  memcpy(w.hw->buf[w.lane] + 8, &b, sizeof(T));
  w.hw->barrier();
  const int g = w.lane >> 4, c = w.lane & 15;
  for (int v = 0; v < 4; ++v) {
    const int row = sizeof(T) == 8 ? g + 4 * v : 4 * g + v;
    T acc = d[v];
    for (int k = 0; k < 4; ++k) {
      T av, bv;
      memcpy(&av, w.hw->buf[k * 16 + row], sizeof(T));
      memcpy(&bv, w.hw->buf[k * 16 + c] + 8, sizeof(T));
      acc = std::fma(av, bv, acc);
    }
    d[v] = acc;
  }
  w.hw->barrier();
}

inline bool wuni(const Wv&, bool b) { return b; }
template <typename T>
inline T wu(const Wv&, T v) { return v; }

template <typename T, int n>
inline void wgather(const Wv& w, T v, T* out) {
  memcpy(w.hw->buf[w.lane], &v, sizeof(T));
  w.hw->barrier();
  for (int i = 0; i < n; ++i) memcpy(&out[i], w.hw->buf[i], sizeof(T));
  w.hw->barrier();
}

// butterfly reductions, same partners and association as the device (own + partner at every level)
template <typename T, typename Op>
inline T host_butterfly(const Wv& w, T v, Op op) {
  memcpy(w.hw->buf[w.lane], &v, sizeof(T));
  w.hw->barrier();
  T vals[WL];
  for (int l = 0; l < WL; ++l) memcpy(&vals[l], w.hw->buf[l], sizeof(T));
  w.hw->barrier();
  // the device's partners in the device's order (mr_wave_prims.h wreduce): xor 1, xor 2,
  // half-row mirror, row mirror, xor 16, xor 32
  for (int lev = 0; lev < 6; ++lev) {
    T nv[WL];
    for (int l = 0; l < WL; ++l) {
      const int p = lev == 0 ? l ^ 1 : lev == 1 ? l ^ 2 : lev == 2 ? (l & ~7) | (7 - (l & 7))
                  : lev == 3 ? (l & ~15) | (15 - (l & 15)) : lev == 4 ? l ^ 16 : l ^ 32;
      nv[l] = op(vals[l], vals[p]);
    }
    for (int l = 0; l < WL; ++l) vals[l] = nv[l];
  }
  return vals[w.lane];
}
template <typename T>
inline T wsum(const Wv& w, T v) { return host_butterfly(w, v, [](T a, T b) { return a + b; }); }
template <typename T>
inline T wmax(const Wv& w, T v) { return host_butterfly(w, v, [](T a, T b) { return b > a ? b : a; }); }
template <typename T>
inline T wmin(const Wv& w, T v) { return host_butterfly(w, v, [](T a, T b) { return b < a ? b : a; }); }
inline bool wany(const Wv& w, bool b) { return wmax(w, b ? 1 : 0) != 0; }
inline bool wall(const Wv& w, bool b) { return wmin(w, b ? 1 : 0) != 0; }

// Run body(hw, lane, arg) as 64 fibers to completion.
inline void host_wave_run(HostWave& hw, void (*body)(HostWave*, int, void*), void* arg) {
  const size_t ss = 512 * 1024;
  hw.stacks = (char*)malloc(ss * WL);
  hw.body = body;
  hw.arg = arg;
  hw.cur = hw.arrived = hw.done = 0;
  struct Entry {
    static void run(int lo, int hi) {
      HostWave* h = (HostWave*)(((uintptr_t)(unsigned)hi << 32) | (uintptr_t)(unsigned)lo);
      const int lane = h->cur;
      h->body(h, lane, h->arg);
      h->fin[lane] = 1;
      h->done++;
    }
  };
  const uintptr_t p = (uintptr_t)&hw;
  for (int l = 0; l < WL; ++l) {
    hw.fin[l] = 0;
    getcontext(&hw.ctx[l]);
    hw.ctx[l].uc_stack.ss_sp = hw.stacks + ss * l;
    hw.ctx[l].uc_stack.ss_size = ss;
    hw.ctx[l].uc_link = &hw.main_ctx;
    makecontext(&hw.ctx[l], (void (*)())Entry::run, 2, (int)(unsigned)(p & 0xffffffffu), (int)(unsigned)(p >> 32));
  }
  // Fiber 0 starts; barriers rotate through (and thereby start) the others.  Control comes back
  // here only when a fiber returns: then every other fiber has passed its last barrier (uniform
  // barrier sequence) or has not started, and may simply be resumed.
  hw.cur = WL - 1;
  while (hw.done < WL) {
    int next = -1;
    for (int l = 0; l < WL; ++l) {
      const int c = (hw.cur + 1 + l) % WL;
      if (!hw.fin[c]) { next = c; break; }
    }
    if (next < 0) break;
    hw.cur = next;
    swapcontext(&hw.main_ctx, &hw.ctx[next]);
  }
  free(hw.stacks);
  hw.stacks = nullptr;
}

template <typename T>
inline const T* wu_ptr(const T* p) { return p; }
template <typename T>
inline T* wu_gptr(T* p) { return p; }
template <typename T>
inline T* wu_any(T* p) { return p; }

template <typename T>
struct WBuf {
  T* p;
  WBuf(T* base, unsigned) : p(base) {}
  T ld(unsigned uoff, unsigned loff) const { return p[uoff + loff]; }
  void st(T x, unsigned uoff, unsigned loff) const { p[uoff + loff] = x; }
};

// host emulation of wtranspose4 (same result: lane (g, c) gets register g of lane (s, c))
template <typename T>
inline void wtranspose4(const Wv& w, T* d) {
  const int g = w.lane >> 4, c = w.lane & 15;
  T out[4];
  for (int s = 0; s < 4; ++s) {
    T t[4];
    for (int r = 0; r < 4; ++r) t[r] = wshfl(w, d[r], s * 16 + c);
    out[s] = t[g];
  }
  for (int s = 0; s < 4; ++s) d[s] = out[s];
}

#endif

}  // namespace mr
