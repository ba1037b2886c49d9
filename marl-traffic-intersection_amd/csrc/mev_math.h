// mev_math.h — bit-exact replicas of the glibc 2.35 float libm routines the
// reference simulator calls, usable on the gfx950 device and on the host.
//
// Why: the reference (cpp/Car.cpp, cpp/Lidar.cpp, cpp/IntersectionEnv.cpp,
// cpp/TrafficFlow.cpp) is compiled against glibc, whose sinf/cosf/tanf/atan2f
// are NOT correctly rounded (SURVEY.md §7.3 hard part 1).  A device trig that
// differs by one ulp flips `int(cx + dx*dist)` in the LiDAR march and, through
// trajectory chaos, every later observation.  So the device path evaluates the
// SAME algorithms glibc 2.35 evaluates, operation for operation:
//
//   mev_sincosf  — glibc sysdeps/ieee754/flt-32 sincosf (optimized-routines):
//                  double-precision polynomial, reduce_fast below 120, the
//                  192-bit 4/pi table above.  glibc's x86-64 ifunc picks the
//                  FMA build on FMA hosts; MEV_SINCOS_FMA selects which
//                  contraction pattern is reproduced (tests/test_devmath.py
//                  checks both against the host libm and pins the choice).
//   mev_tanf     — glibc 2.35 tanf: sincosf-style reduction + fdlibm __kernel_tanf.
//   mev_atan2f   — fdlibm e_atan2f + s_atanf (11-term polynomial).
//   mev_hypotf   — glibc 2.35 hypotf: (float)sqrt((double)x*x + (double)y*y).
//   mev_fmodf    — exact remainder (any correct fmodf is bit-identical).
//
// Every constant below was checked against the tables in this image's
// /lib/x86_64-linux-gnu/libm.so.6 and every function is compared bit-for-bit
// with that libm over the argument ranges the simulator uses (tests/test_devmath.py).
// All code must be compiled with -ffp-contract=off.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MEV_HD __host__ __device__ inline
#else
#include <math.h>
#define MEV_HD static inline
#endif

#ifndef MEV_SINCOS_FMA
#define MEV_SINCOS_FMA 1
#endif

namespace mev {

MEV_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
MEV_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
MEV_HD uint64_t d2u(double d) { return __builtin_bit_cast(uint64_t, d); }

MEV_HD double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }
MEV_HD float fabs_f(float x) { return u2f(f2u(x) & 0x7fffffffu); }

// a + b*c in double, contracted or not (glibc FMA vs generic build).
template <bool FMA>
MEV_HD double madd(double a, double b, double c) {
    if constexpr (FMA) return fma_d(b, c, a);
    else return a + b * c;
}

// ---------------------------------------------------------------- sincosf ---
struct SinCosTab {
    double sign[4];
    double hpi_inv;
    double hpi;
    double c0, c1, s1, c2, s2, c3, s3, c4;
};

static constexpr SinCosTab kSinCos[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
     0x1p+0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
     -0x1p+0, 0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16},
};

static constexpr uint32_t kInvPio4[24] = {
    0xa2u,       0xa2f9u,     0xa2f983u,   0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u,
    0x6e4e4415u, 0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
    0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u,
    0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u,
};

MEV_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ffu; }

template <bool FMA>
MEV_HD void sincosf_poly(double x, double x2, const SinCosTab& p, int n, float* sinp, float* cosp) {
    const double x4 = x2 * x2;
    const double x3 = x2 * x;
    const double c2 = madd<FMA>(p.c3, x2, p.c4);
    const double s1 = madd<FMA>(p.s2, x2, p.s3);
    const double c1 = madd<FMA>(p.c0, x2, p.c1);
    const double x5 = x3 * x2;
    const double x6 = x4 * x2;
    const double s = madd<FMA>(x, x3, p.s1);
    const double c = madd<FMA>(c1, x4, p.c2);
    const float sv = (float)madd<FMA>(s, x5, s1);
    const float cv = (float)madd<FMA>(c, x6, c2);
    if (n & 1) { *sinp = cv; *cosp = sv; }
    else { *sinp = sv; *cosp = cv; }
}

template <bool FMA>
MEV_HD double reduce_fast(double x, const SinCosTab& p, int* np) {
    const double r = x * p.hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    if constexpr (FMA) return fma_d(-(double)n, p.hpi, x);
    else return x - n * p.hpi;
}

MEV_HD double reduce_large(uint32_t xi, int* np) {
    const uint32_t* arr = &kInvPio4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    uint64_t res0 = xi * arr[0];
    const uint64_t res1 = (uint64_t)xi * arr[4];
    const uint64_t res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * 0x1.921fb54442d18p-62;
}

// glibc's polynomial step after a reduction to x (double) and n: with the
// table selector q (n, or n + sign in the large path) sign[q & 3] = {1, -1, -1, 1}
// multiplies x by +-1 (an exact negation) and kSinCos[1] is kSinCos[0] with
// the cosine coefficients c0..c4 negated, so its cosine polynomial -- and the
// rounded float -- is exactly the negation of kSinCos[0]'s; no per-lane table
// loads.  Returns (sin, cos) before the |y| < 2^-12 shortcut.
template <bool FMA>
MEV_HD void sincos_tail(double x, int n, int q, float* so, float* co) {
    // (an exact negation: the sign bit of the high word flipped)
    const double xs = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, x) ^ ((uint64_t)((q + 1) & 2) << 62));
    const SinCosTab& p = kSinCos[0];
    const double x2 = x * x;
    const double x4 = x2 * x2;
    const double x3 = x2 * xs;
    const double c2 = madd<FMA>(p.c3, x2, p.c4);
    const double s1 = madd<FMA>(p.s2, x2, p.s3);
    const double c1 = madd<FMA>(p.c0, x2, p.c1);
    const double x5 = x3 * x2;
    const double x6 = x4 * x2;
    const double sp = madd<FMA>(xs, x3, p.s1);
    const double cp = madd<FMA>(c1, x4, p.c2);
    const float sv = (float)madd<FMA>(sp, x5, s1);
    float cv = (float)madd<FMA>(cp, x6, c2);
    cv = u2f(f2u(cv) ^ ((uint32_t)(q & 2) << 30));
    *so = (n & 1) ? cv : sv;
    *co = (n & 1) ? sv : cv;
}

template <bool FMA>
MEV_HD void sincosf_impl(float y, float* sinp, float* cosp) {
    double x = y;
    int n;
    const SinCosTab* p = &kSinCos[0];
    if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {
        const double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) {
            *sinp = y;
            *cosp = 1.0f;
            return;
        }
        sincosf_poly<FMA>(x, x2, *p, 0, sinp, cosp);
    } else if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast<FMA>(x, *p, &n);
        sincos_tail<FMA>(x, n, n, sinp, cosp);
    } else if (abstop12(y) < abstop12(__builtin_inff())) {
        const uint32_t xi = f2u(y);
        const int sign = xi >> 31;
        x = reduce_large(xi, &n);
        sincos_tail<FMA>(x, n, n + sign, sinp, cosp);
    } else {
        *sinp = *cosp = y - y;  // NaN for inf / NaN input
    }
}


// Same results as sincosf for every finite |y| < 120 with one code path: below
// pi/4 reduce_fast yields n = 0 and x unchanged, so the reduced polynomial is
// glibc's small-argument one; the |y| < 2^-12 shortcut becomes a select --
// checked for every float |y| <= 8 by tests/native/devmath_check.cpp.  A wave
// of beams then does not evaluate the polynomial twice.
template <bool FMA>
MEV_HD void sincosf_below120_impl(float y, float* sinp, float* cosp) {
    int n;
    const double x = reduce_fast<FMA>((double)y, kSinCos[0], &n);
    float so, co;
    sincos_tail<FMA>(x, n, n, &so, &co);
    const bool tiny = abstop12(y) < abstop12(0x1p-12f);  // glibc's shortcut (keeps the sign of -0)
    *sinp = tiny ? y : so;
    *cosp = tiny ? 1.0f : co;
}

template <bool FMA>
MEV_HD void sincosf_reduced_impl(float y, float* sinp, float* cosp) {
    if (!(abstop12(y) < abstop12(120.0f))) {
        sincosf_impl<FMA>(y, sinp, cosp);
        return;
    }
    sincosf_below120_impl<FMA>(y, sinp, cosp);
}

// the simulator's sincosf (glibc results; single path below 120)
MEV_HD void sincosf(float y, float* s, float* c) { sincosf_reduced_impl<MEV_SINCOS_FMA != 0>(y, s, c); }
// the same for a caller that guarantees |y| < 120 (no branch: straight-line code
// the compiler can interleave with other independent work)
MEV_HD void sincosf_below120(float y, float* s, float* c) { sincosf_below120_impl<MEV_SINCOS_FMA != 0>(y, s, c); }

// ------------------------------------------------------------------ tanf ---
MEV_HD float kernel_tanf(float x, float y, int iy) {
    constexpr float one = 1.0f;
    constexpr float pio4 = 7.8539812565e-01f;    // 0x3f490fda
    constexpr float pio4lo = 3.7748947079e-08f;  // 0x33222168
    const float T0 = u2f(0x3eaaaaabu), T1 = u2f(0x3e088889u), T2 = u2f(0x3d5d0dd1u), T3 = u2f(0x3cb327a4u),
                T4 = u2f(0x3c11371fu), T5 = u2f(0x3b6b6916u), T6 = u2f(0x3abede48u), T7 = u2f(0x3a1a26c8u),
                T8 = u2f(0x398137b9u), T9 = u2f(0x38a3f445u), T10 = u2f(0x3895c07au), T11 = u2f(0xb79bae5fu),
                T12 = u2f(0x37d95384u);
    float z, r, v, w, s;
    const int32_t hx = (int32_t)f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix < 0x39000000) {
        if ((int)x == 0) {
            if ((ix | (iy + 1)) == 0) return one / fabs_f(x);
            else if (iy == 1) return x;
            else return -one / x;
        }
    }
    if (ix >= 0x3f2ca140) {
        if (hx < 0) { x = -x; y = -y; }
        z = pio4 - x;
        w = pio4lo - y;
        x = z + w;
        y = 0.0f;
        if (fabs_f(x) < 0x1p-13f) return (float)((1 - ((hx >> 30) & 2)) * iy) * (1.0f - (float)(2 * iy) * x);
    }
    z = x * x;
    w = z * z;
    r = T1 + w * (T3 + w * (T5 + w * (T7 + w * (T9 + w * T11))));
    v = z * (T2 + w * (T4 + w * (T6 + w * (T8 + w * (T10 + w * T12)))));
    s = z * x;
    r = y + z * (s * (r + v) + y);
    r += T0 * s;
    w = x + r;
    if (ix >= 0x3f2ca140) {
        v = (float)iy;
        return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
    }
    if (iy == 1) return w;
    float a, t;
    z = u2f(f2u(w) & 0xfffff000u);
    v = r - (z - x);
    t = a = -1.0f / w;
    t = u2f(f2u(t) & 0xfffff000u);
    s = 1.0f + t * z;
    return t + a * (s + t * v);
}

MEV_HD float tanf(float x) {
    const uint32_t ix = f2u(x) & 0x7fffffffu;
    if (ix <= 0x3f490fdau) return kernel_tanf(x, 0.0f, 1);
    if (ix >= 0x7f800000u) return x - x;
    int n;
    double xd;
    if (abstop12(x) < abstop12(120.0f)) {
        // glibc 2.35 s_tanf.c: reduce_fast without the FMA build (tanf is not an ifunc).
        const double r = (double)x * 0x1.45f306dc9c883p+23;
        n = ((int32_t)r + 0x800000) >> 24;
        xd = (double)x - (double)n * 0x1.921fb54442d18p+0;
    } else {
        const uint32_t xi = f2u(x);
        xd = reduce_large(xi, &n);
        if (xi >> 31) { xd = -xd; n = -n; }
    }
    const float y0 = (float)xd;
    const float y1 = (float)(xd - (double)y0);
    return kernel_tanf(y0, y1, 1 - ((n & 1) << 1));
}

// ----------------------------------------------------------------- atanf ---
MEV_HD float atanf(float x) {
    const float atanhi0 = u2f(0x3eed6338u), atanhi1 = u2f(0x3f490fdau), atanhi2 = u2f(0x3f7b985eu),
                atanhi3 = u2f(0x3fc90fdau);
    const float atanlo0 = u2f(0x31ac3769u), atanlo1 = u2f(0x33222168u), atanlo2 = u2f(0x33140fb4u),
                atanlo3 = u2f(0x33a22168u);
    const float aT0 = u2f(0x3eaaaaabu), aT1 = u2f(0xbe4ccccdu), aT2 = u2f(0x3e124925u), aT3 = u2f(0xbde38e38u),
                aT4 = u2f(0x3dba2e6eu), aT5 = u2f(0xbd9d8795u), aT6 = u2f(0x3d886b35u), aT7 = u2f(0xbd6ef16bu),
                aT8 = u2f(0x3d4bda59u), aT9 = u2f(0xbd15a221u), aT10 = u2f(0x3c8569d7u);
    constexpr float one = 1.0f;
    float w, s1, s2, z, hi = 0.0f, lo = 0.0f;
    const int32_t hx = (int32_t)f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = fabs_f(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - one) / (2.0f + x); hi = atanhi0; lo = atanlo0; }
            else { id = 1; x = (x - one) / (x + one); hi = atanhi1; lo = atanlo1; }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (one + 1.5f * x); hi = atanhi2; lo = atanlo2; }
            else { id = 3; x = -1.0f / x; hi = atanhi3; lo = atanlo3; }
        }
    }
    z = x * x;
    w = z * z;
    s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    z = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -z : z;
}

MEV_HD float atan2f(float y, float x) {
    constexpr float tiny = 1.0e-30f;
    const float pi_o_4 = u2f(0x3f490fdbu), pi_o_2 = u2f(0x3fc90fdbu), pi = u2f(0x40490fdbu),
                pi_lo = u2f(0xb3bbbd2eu);
    float z;
    const int32_t hx = (int32_t)f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)f2u(y);
    const int32_t iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        } else {
            switch (m) {
                case 0: return 0.0f;
                case 1: return -0.0f;
                case 2: return pi + tiny;
                default: return -pi - tiny;
            }
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = atanf(fabs_f(y / x));
    switch (m) {
        case 0: return z;
        case 1: return u2f(f2u(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// Branch-free forms of atanf / atan2f for wave code: the same operations in the
// same order as above, with fdlibm's range reduction chosen by selects instead
// of branches -- in a wave whose lanes fall into different ranges or quadrants
// the branchy form runs every taken path one after another.  The reduction's
// four quotients are one (p*|x| - q) / (r + s*|x|):
//   id 0: (2|x| - 1) / (2 + |x|)   id 1: (|x| - 1) / (1 + |x|)
//   id 2: (|x| - 1.5) / (1 + 1.5|x|)   id 3: (0|x| - 1) / (0 + |x|) = -1/|x|
// (1*a and 0 + a are exact, addition commutes: the same roundings as fdlibm's).
// atan2f_bf is exact for every input atan2f_special() rejects (zero, infinite
// or NaN operands); tests/native/devmath_check.cpp checks both against glibc.
MEV_HD float atanf_bf(float x) {
    const float atanhi[4] = {u2f(0x3eed6338u), u2f(0x3f490fdau), u2f(0x3f7b985eu), u2f(0x3fc90fdau)};
    const float atanlo[4] = {u2f(0x31ac3769u), u2f(0x33222168u), u2f(0x33140fb4u), u2f(0x33a22168u)};
    const float aT0 = u2f(0x3eaaaaabu), aT1 = u2f(0xbe4ccccdu), aT2 = u2f(0x3e124925u), aT3 = u2f(0xbde38e38u),
                aT4 = u2f(0x3dba2e6eu), aT5 = u2f(0xbd9d8795u), aT6 = u2f(0x3d886b35u), aT7 = u2f(0xbd6ef16bu),
                aT8 = u2f(0x3d4bda59u), aT9 = u2f(0xbd15a221u), aT10 = u2f(0x3c8569d7u);
    const int32_t hx = (int32_t)f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    const float ax = fabs_f(x);
    const bool small = ix < 0x3ee00000;  // id -1: no reduction
    const int id = ix < 0x3f300000 ? 0 : (ix < 0x3f980000 ? 1 : (ix < 0x401c0000 ? 2 : 3));
    const float pp = id == 0 ? 2.0f : (id == 3 ? 0.0f : 1.0f);
    const float qq = id == 2 ? 1.5f : 1.0f;
    const float rr = id == 0 ? 2.0f : (id == 3 ? 0.0f : 1.0f);
    const float ss = id == 2 ? 1.5f : 1.0f;
    const float red = (pp * ax - qq) / (rr + ss * ax);
    const float xr = small ? x : red;
    const float z = xr * xr;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const float hi = id == 0 ? atanhi[0] : (id == 1 ? atanhi[1] : (id == 2 ? atanhi[2] : atanhi[3]));
    const float lo = id == 0 ? atanlo[0] : (id == 1 ? atanlo[1] : (id == 2 ? atanlo[2] : atanlo[3]));
    const float r_small = xr - xr * (s1 + s2);
    const float zz = hi - ((xr * (s1 + s2) - lo) - xr);
    float r = small ? r_small : (hx < 0 ? -zz : zz);
    if (ix < 0x31000000) r = x;                                                   // tiny: atan x = x
    if (ix >= 0x4c000000) r = hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];  // |x| >= 2^25
    return ix > 0x7f800000 ? x + x : r;
}

// operands atan2f_bf does not handle (its caller takes atan2f for the wave)
MEV_HD bool atan2f_special(float y, float x) {
    const uint32_t ax = f2u(x) & 0x7fffffffu, ay = f2u(y) & 0x7fffffffu;
    return ax == 0u || ay == 0u || ax >= 0x7f800000u || ay >= 0x7f800000u;
}

MEV_HD float atan2f_bf(float y, float x) {
    const float pi = u2f(0x40490fdbu), pi_o_2 = u2f(0x3fc90fdbu), pi_lo = u2f(0xb3bbbd2eu);
    const int32_t hx = (int32_t)f2u(x);
    const int32_t ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)f2u(y);
    const int32_t iy = hy & 0x7fffffff;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    const int32_t k = (iy - ix) >> 23;
    float z = atanf_bf(fabs_f(y / x));
    z = (hx < 0 && k < -60) ? 0.0f : z;
    z = k > 60 ? pi_o_2 + 0.5f * pi_lo : z;
    const float r2 = pi - (z - pi_lo), r3 = (z - pi_lo) - pi;
    const float r = m == 0 ? z : (m == 1 ? u2f(f2u(z) ^ 0x80000000u) : (m == 2 ? r2 : r3));
    return hx == 0x3f800000 ? atanf_bf(y) : r;  // x == 1: fdlibm returns atanf(y)
}

// ---------------------------------------------------------------- hypotf ---
MEV_HD float hypotf(float x, float y) {
    // glibc 2.35 e_hypotf.c (finite inputs): one double evaluation, one rounding.
    const double dx = x, dy = y;
    return (float)__builtin_sqrt(dx * dx + dy * dy);
}

// ----------------------------------------------------------------- fmodf ---
// Exact IEEE remainder x - trunc(x/y)*y.  fmod is exact (the result is always
// representable), so any correct method returns glibc's bits; this one is
// branch-light for the GPU: estimate the quotient with a multiply, get the
// remainder exactly with one fma (exact whenever the quotient is right), and
// correct a one-off estimate.  Falls back to the bit-level loop when the
// quotient does not fit in 24 bits.  Checked bit-for-bit against glibc
// (tests/native/devmath_check.cpp).
MEV_HD float fmodf_bits(float x, float y) {  // musl-style reference loop
    uint32_t ux = f2u(x), uy = f2u(y);
    int ex = (ux >> 23) & 0xff;
    int ey = (uy >> 23) & 0xff;
    const uint32_t sx = ux & 0x80000000u;
    uint32_t i;
    if ((uy << 1) == 0 || ex == 0xff || ((uy & 0x7fffffffu) > 0x7f800000u)) return (x * y) / (x * y);
    if ((ux << 1) <= (uy << 1)) {
        if ((ux << 1) == (uy << 1)) return 0.0f * x;
        return x;
    }
    if (!ex) {
        for (i = ux << 9; (int32_t)i >= 0; ex--, i <<= 1) {}
        ux <<= -ex + 1;
    } else {
        ux &= 0xffffffffu >> 9;
        ux |= 1u << 23;
    }
    if (!ey) {
        for (i = uy << 9; (int32_t)i >= 0; ey--, i <<= 1) {}
        uy <<= -ey + 1;
    } else {
        uy &= 0xffffffffu >> 9;
        uy |= 1u << 23;
    }
    for (; ex > ey; ex--) {
        i = ux - uy;
        if ((int32_t)i >= 0) {
            if (i == 0) return 0.0f * x;
            ux = i;
        }
        ux <<= 1;
    }
    i = ux - uy;
    if ((int32_t)i >= 0) {
        if (i == 0) return 0.0f * x;
        ux = i;
    }
    for (; (ux >> 23) == 0; ux <<= 1, ex--) {}
    if (ex > 0) {
        ux -= 1u << 23;
        ux |= (uint32_t)ex << 23;
    } else {
        ux >>= -ex + 1;
    }
    ux |= sx;
    return u2f(ux);
}

MEV_HD float fmodf(float x, float y) {
    const float ax = fabs_f(x), ay = fabs_f(y);
    // fast path: finite, normal y, quotient < 2^23
    if (ay >= 0x1p-100f && ay < 0x1p100f && ax < ay * 0x1p22f) {
        if (ax < ay) return x;
        float q = __builtin_truncf(ax * (1.0f / ay));
        float r = __builtin_fmaf(-q, ay, ax);  // exact when q == trunc(ax/ay)
        if (r < 0.0f) { q -= 1.0f; r = __builtin_fmaf(-q, ay, ax); }
        else if (r >= ay) { q += 1.0f; r = __builtin_fmaf(-q, ay, ax); }
        return u2f(f2u(r) | (f2u(x) & 0x80000000u));  // result carries the sign of x (also for zero)
    }
    return fmodf_bits(x, y);
}

}  // namespace mev
