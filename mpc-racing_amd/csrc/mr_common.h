// Common definitions of the batched racing-MPC solver (host + gfx950 device).
//
// One source is compiled twice: by hipcc for gfx950 (the product,
// libmpcracing.so) and by g++ (libmpcracing_host.so, used only by the CPU
// tests to check the solver logic without a GPU).
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MR_HD __host__ __device__ __forceinline__
#define MR_DEVICE_BUILD 1
#else
#define MR_HD inline
#define MR_DEVICE_BUILD 0
#endif

namespace mr {

MR_HD double mr_sin(double a) { return sin(a); }
MR_HD double mr_cos(double a) { return cos(a); }
MR_HD double mr_tan(double a) { return tan(a); }
MR_HD double mr_atan(double a) { return atan(a); }
MR_HD double mr_atan2(double y, double x) { return atan2(y, x); }
MR_HD double mr_sqrt(double a) { return sqrt(a); }
MR_HD double mr_exp(double a) { return exp(a); }
MR_HD double mr_log(double a) { return log(a); }
MR_HD double mr_abs(double a) { return fabs(a); }
MR_HD float mr_sin(float a) { return sinf(a); }
MR_HD float mr_cos(float a) { return cosf(a); }
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MR_LIBM_F32)
// fp32 on the device, for the model's steering and slip angles (|a| < 1.6 rad): tan from the hardware
// sine / cosine (the library tanf carries a ~140-instruction large-argument reduction), atan2 by an
// odd degree-15 polynomial on [0, 1] with octant reduction (max error 1.3e-7 rad, ~2 ulp, vs ~45
// instructions with a division for the library's).  fp64 and the host build keep libm.
MR_HD float mr_tan(float a) { return __sinf(a) * __builtin_amdgcn_rcpf(__cosf(a)); }
MR_HD float mr_atan2(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  const float q = mx > 0.0f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
  const float s = q * q;
  float p = -0.004073309246450663f;
  p = p * s + 0.021946610882878304f;
  p = p * s - 0.056063175201416016f;
  p = p * s + 0.09656256437301636f;
  p = p * s - 0.13915802538394928f;
  p = p * s + 0.19948509335517883f;
  p = p * s - 0.3333010673522949f;
  p = p * s + 0.999999463558197f;
  float r = q * p;
  r = ay > ax ? 1.5707963267948966f - r : r;
  r = x < 0.0f ? 3.141592653589793f - r : r;
  return copysignf(r, y);
}
#else
MR_HD float mr_tan(float a) { return tanf(a); }
MR_HD float mr_atan2(float y, float x) { return atan2f(y, x); }
#endif
MR_HD float mr_atan(float a) { return atanf(a); }
MR_HD float mr_sqrt(float a) { return sqrtf(a); }
MR_HD float mr_exp(float a) { return expf(a); }
#if MR_DEVICE_BUILD
// fp32 ln on the device: the hardware log2 (v_log_f32) times ln 2 -- 2 instructions against the library's
// 8 (its extended-precision ln 2 product and infinity guard); a ~2 ulp result for the barrier terms
// (fp32 solves only; -inf at 0 and NaN below, as logf)
MR_HD float mr_log(float a) { return __builtin_amdgcn_logf(a) * 0.69314718055994531f; }
#else
MR_HD float mr_log(float a) { return logf(a); }
#endif
MR_HD float mr_abs(float a) { return fabsf(a); }

// 1/sqrt(a), a > 0: IEEE in fp64 and on the host; the hardware v_rsq_f32 (1 ulp) on the device
// in fp32 (the pivots of the Riccati sweep, on its serial critical path)
MR_HD double mr_rsqrt(double a) { return 1.0 / sqrt(a); }
#if MR_DEVICE_BUILD
MR_HD float mr_rsqrt(float a) { return __builtin_amdgcn_rsqf(a); }
// keep a value computed in every lane (stops the compiler sinking it into per-lane branches)
#define MR_MATERIALIZE(x) __asm__ volatile("" : "+v"(x))
#else
MR_HD float mr_rsqrt(float a) { return 1.0f / sqrtf(a); }
#define MR_MATERIALIZE(x) ((void)0)
#endif

template <typename T> MR_HD T mr_max(T a, T b) { return a > b ? a : b; }
template <typename T> MR_HD T mr_min(T a, T b) { return a < b ? a : b; }
// machine epsilon of the solve precision (IPOPT's Compare_le tolerance 10 eps |ref|)
template <typename T> MR_HD constexpr T mr_eps() { return sizeof(T) == 8 ? T(2.220446049250313e-16) : T(1.1920928955078125e-07); }

// models/VehicleParameters.py:3-41 (runtime values so a caller may change them,
// as the reference's class attributes can be).
template <typename T>
struct VehParams {
  T m, Iz, lf, lr, Cf, Cr, T_max, r_wheel, C_wheel, R, rho, C_d, A_f, C_roll, g, max_steer,
      Vblendmin, Vblendmax;
};

// Value and first/second derivative of a scalar lateral-force law at a slip angle.
template <typename T>
struct TyreJet {
  T v, d, dd;
};

// Cancellation-free constants of the Pacejka magic formula (learning/vehicle.py:79-92),
// computed once on the host in fp64: Fy(a) = BCD*phi*h(B*phi), phi = a*(1 + E*(atan(Ba)/(Ba) - 1)).
template <typename T>
struct TyreCoef {
  T B, C, E, BCD, K2;  // K2 = E*B*B
};

// Second-order jet (value, d/da, d2/da2) arithmetic for the tyre law.
template <typename T>
struct Jet2 {
  T v, d, dd;
};
template <typename T> MR_HD Jet2<T> jmul(Jet2<T> a, Jet2<T> b) {
  return {a.v * b.v, a.d * b.v + a.v * b.d, a.dd * b.v + T(2) * a.d * b.d + a.v * b.dd};
}
template <typename T> MR_HD Jet2<T> jadd(Jet2<T> a, Jet2<T> b) { return {a.v + b.v, a.d + b.d, a.dd + b.dd}; }
template <typename T> MR_HD Jet2<T> jscale(Jet2<T> a, T s) { return {a.v * s, a.d * s, a.dd * s}; }
template <typename T> MR_HD Jet2<T> jaddc(Jet2<T> a, T c) { return {a.v + c, a.d, a.dd}; }
// apply a scalar function with value f0, derivative f1, second derivative f2 at a.v
template <typename T> MR_HD Jet2<T> japply(Jet2<T> a, T f0, T f1, T f2) {
  return {f0, f1 * a.d, f2 * a.d * a.d + f1 * a.dd};
}

// Pacejka lateral force with derivatives (stable form; series near 0 where the
// learned coefficients live: |B*alpha| ~ 1e-7, |E| ~ 1e10).
template <typename T>
MR_HD TyreJet<T> pacejka_jet(const TyreCoef<T>& c, T alpha) {
  Jet2<T> a{alpha, T(1), T(0)};
  Jet2<T> x = jscale(a, c.B);
  Jet2<T> eg;
  if (mr_abs(x.v) < T(1e-3)) {
    Jet2<T> x2 = jmul(x, x);
    // E*(atan(x)/x - 1) = K2*a^2*(-1/3 + x^2/5 - x^4/7)
    Jet2<T> poly = jaddc(jmul(x2, jaddc(jscale(x2, T(-1.0 / 7.0)), T(1.0 / 5.0))), T(-1.0 / 3.0));
    eg = jscale(jmul(jmul(a, a), poly), c.K2);
  } else {
    T xv = x.v;
    T at = mr_atan(xv);
    T q = T(1) / (T(1) + xv * xv);
    // g(x) = atan(x)/x - 1 ; g' = (q x - atan)/x^2 ; g'' = (-2 q^2 x^2 - 2(q x - atan)... ) computed directly
    T g0 = at / xv - T(1);
    T g1 = (q * xv - at) / (xv * xv);
    T dq = T(-2) * xv * q * q;
    T g2 = ((dq * xv + q - q) * xv * xv - T(2) * xv * (q * xv - at)) / (xv * xv * xv * xv);
    eg = jscale(japply(x, g0, g1, g2), c.E);
  }
  Jet2<T> phi = jmul(a, jaddc(eg, T(1)));
  Jet2<T> y = jscale(phi, c.B);
  Jet2<T> h;
  if (mr_abs(y.v) < T(1e-3)) {
    T c2 = c.C * c.C;
    Jet2<T> y2 = jmul(y, y);
    h = jaddc(jmul(y2, jaddc(jscale(y2, T(1.0 / 5.0) + c2 / T(6) + c2 * c2 / T(120)), -(T(1.0 / 3.0) + c2 / T(6)))), T(1));
  } else {
    // h(y) = sin(C atan y)/(C y)
    T yv = y.v;
    T at = mr_atan(yv);
    T s = mr_sin(c.C * at), co = mr_cos(c.C * at);
    T q = T(1) / (T(1) + yv * yv);
    T num = s, dnum = co * c.C * q;
    T d2num = -s * c.C * c.C * q * q + co * c.C * (T(-2) * yv * q * q);
    T den = c.C * yv, dden = c.C;
    T h0 = num / den;
    T h1 = (dnum * den - num * dden) / (den * den);
    T h2 = (d2num * den * den - T(2) * dnum * dden * den + T(2) * num * dden * dden) / (den * den * den);
    h = japply(y, h0, h1, h2);
  }
  Jet2<T> fy = jscale(jmul(phi, h), c.BCD);
  return {fy.v, fy.d, fy.dd};
}

}  // namespace mr
