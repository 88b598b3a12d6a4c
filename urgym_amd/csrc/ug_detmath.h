/* ug_detmath.h -- deterministic double-precision elementary functions.
 *
 * Why: the HIP kernels and the CPU restatement (oracle/) must produce
 * bit-identical trajectories, so neither may call its platform libm (glibc and
 * ROCm's OCML differ in the last ulp).  Everything below is built only from
 * IEEE-754 correctly-rounded +, -, *, /, sqrt and rint, which x86-64 SSE2 and
 * gfx950 both implement exactly; both sides compile with -ffp-contract=off so
 * no FMA is formed behind our back.
 *
 * Algorithms and coefficients follow the freely-redistributable Sun fdlibm
 * 5.3 (s_sin.c/k_sin.c/k_cos.c, s_atan.c, e_atan2.c, e_asin.c, e_acos.c,
 * e_exp.c, s_expm1.c, s_tanh.c); accuracy <= 1-2 ulp on the ranges used
 * (|x| < 1e5 for sin/cos).  Usable from C99 (gcc) and HIP device code.  Pinned from outside by
 * tests/test_detmath_kat.py: <= 1 ulp from an extended-precision reference for sin, cos, atan, asin, acos and expm1,
 * <= 2 ulp for tanh and atan2 (fdlibm's own bound, measured 1.93 / 1.42; numpy's tanh, which the reference's reward
 * calls, is within ~1.1).
 */
#ifndef UG_DETMATH_H
#define UG_DETMATH_H

#ifdef __HIPCC__
#define UG_HD __host__ __device__ static inline
#else
#define UG_HD static inline
#include <math.h>
#endif

#include <stdint.h>

typedef union { double d; uint64_t u; } ug_dbits;

UG_HD double ug_fabs(double x) { return x < 0.0 ? -x : x; }
UG_HD double ug_sqrt(double x) { return __builtin_sqrt(x); }
UG_HD double ug_rint(double x) { return __builtin_rint(x); }
UG_HD double ug_min(double a, double b) { return a < b ? a : b; }
UG_HD double ug_max(double a, double b) { return a > b ? a : b; }
UG_HD double ug_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
/* btClamp(v, -m, m) as btMultiBody::applyDeltaVeeMultiDof applies it to every dof velocity [ext] (a NaN passes) */
UG_HD double ug_vclamp(double v, double m) { return v < -m ? -m : (m < v ? m : v); }
/* numpy.linalg.norm of a 3-vector as this image's numpy computes it (OpenBLAS ddot: fused
 * multiply-adds in element order, then sqrt) -- checked against numpy in tests/test_oracle_kat.py */
UG_HD double ug_norm3(double x, double y, double z) { return __builtin_sqrt(__builtin_fma(z, z, __builtin_fma(y, y, x * x))); }
UG_HD double ug_trunc_lo(double x) { ug_dbits b; b.d = x; b.u &= 0xffffffff00000000ULL; return b.d; }
UG_HD double ug_scalbn(double x, int k) {
    /* x * 2^k for |k| <= 1022, exact */
    ug_dbits b; b.u = (uint64_t)(k + 1023) << 52; return x * b.d;
}

#define UG_PI 3.14159265358979311600e+00
#define UG_PI_LO 1.22464679914735317720e-16
#define UG_PIO2_HI 1.57079632679489655800e+00
#define UG_PIO2_LO 6.12323399573676603587e-17

/* ---- sin / cos ---- */
UG_HD double ug__ksin(double x, double y) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x, w = z * z;
    double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    double v = z * x;
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
UG_HD double ug__kcos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x, w = z * z;
    double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    double hz = 0.5 * z;
    w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}
/* reduce x to y0+y1 in [-pi/4, pi/4], return quadrant */
UG_HD int ug__rem_pio2(double x, double* y0, double* y1) {
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21;
    double fn = ug_rint(x * invpio2);
    double r = x - fn * pio2_1;
    double w = fn * pio2_1t;
    double t = r;
    /* second stage (fdlibm medium case) for extra bits */
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    double yy0 = r - w;
    *y0 = yy0;
    *y1 = (r - yy0) - w;
    /* the quadrant fn mod 4, exact for every integer-valued fn: (int)fn is undefined past 2^31 (x86 returns INT_MIN,
     * gfx950 saturates), which made a runaway state's angles differ between the two builds; NaN gives quadrant 0 */
    const double q4 = fn - 4.0 * __builtin_floor(fn * 0.25);
    return q4 >= 0.0 && q4 < 4.0 ? (int)q4 : 0;
}
UG_HD double ug_sin(double x) {
    if (ug_fabs(x) <= 7.85398163397448278999e-01) return ug__ksin(x, 0.0);
    double y0, y1;
    int n = ug__rem_pio2(x, &y0, &y1);
    switch (n & 3) {
        case 0: return ug__ksin(y0, y1);
        case 1: return ug__kcos(y0, y1);
        case 2: return -ug__ksin(y0, y1);
        default: return -ug__kcos(y0, y1);
    }
}
UG_HD double ug_cos(double x) {
    if (ug_fabs(x) <= 7.85398163397448278999e-01) return ug__kcos(x, 0.0);
    double y0, y1;
    int n = ug__rem_pio2(x, &y0, &y1);
    switch (n & 3) {
        case 0: return ug__kcos(y0, y1);
        case 1: return -ug__ksin(y0, y1);
        case 2: return -ug__kcos(y0, y1);
        default: return ug__ksin(y0, y1);
    }
}

/* sin and cos together, branch-free: the same kernels on the same reduced argument as ug_sin / ug_cos (the
 * small-argument path as a select), so the results are identical to theirs */
UG_HD void ug_sincos(double x, double* sn, double* cs) {
    double r0, r1;
    int nr = ug__rem_pio2(x, &r0, &r1);
    const int small = ug_fabs(x) <= 7.85398163397448278999e-01;
    const double y0 = small ? x : r0, y1 = small ? 0.0 : r1;
    const int q = (small ? 0 : nr) & 3;
    const double ks = ug__ksin(y0, y1), kc = ug__kcos(y0, y1);
    *sn = q == 0 ? ks : (q == 1 ? kc : (q == 2 ? -ks : -kc));
    *cs = q == 0 ? kc : (q == 1 ? -ks : (q == 2 ? -kc : ks));
}

/* ---- atan / atan2 ---- */
UG_HD double ug_atan(double x) {
    const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                              9.82793723247329054082e-01, 1.57079632679489655800e+00};
    const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                              1.39033110312309984516e-17, 6.12323399573676603587e-17};
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    int neg = x < 0.0;
    double ax = ug_fabs(x);
    int id;
    if (ax >= 7.378697629483821e19) return neg ? -(atanhi[3] + atanlo[3]) : (atanhi[3] + atanlo[3]);
    if (ax < 0.4375) {
        if (ax < 3.725290298461914e-09) return x;
        id = -1;
    } else if (ax < 1.1875) {
        if (ax < 0.6875) { id = 0; ax = (2.0 * ax - 1.0) / (2.0 + ax); }
        else { id = 1; ax = (ax - 1.0) / (ax + 1.0); }
    } else if (ax < 2.4375) { id = 2; ax = (ax - 1.5) / (1.0 + 1.5 * ax); }
    else { id = 3; ax = -1.0 / ax; }
    double z = ax * ax, w = z * z;
    double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((ax * (s1 + s2) - atanlo[id]) - ax);
    return neg ? -z : z;
}
UG_HD double ug_atan2(double y, double x) {
    if (x == 1.0) return ug_atan(y);
    int m = (y < 0.0 || (y == 0.0 && 1.0 / y < 0.0)) | (2 * (x < 0.0 || (x == 0.0 && 1.0 / x < 0.0)));
    if (y == 0.0) {
        if (m < 2) return y;
        return m == 2 ? UG_PI : -UG_PI;
    }
    if (x == 0.0) return y < 0.0 ? -UG_PIO2_HI - UG_PIO2_LO : UG_PIO2_HI + UG_PIO2_LO;
    if (ug_fabs(x) == __builtin_inf() && ug_fabs(y) == __builtin_inf()) { /* e_atan2.c: both infinite */
        const double pio4 = 7.8539816339744827900e-01;
        return m == 0 ? pio4 : (m == 1 ? -pio4 : (m == 2 ? 3.0 * pio4 : -3.0 * pio4));
    }
    double q = ug_fabs(y / x), z;
    if (q > 1.152921504606847e18) z = UG_PIO2_HI + 0.5 * UG_PI_LO;
    else if (x < 0.0 && q < 8.673617379884035e-19) z = 0.0;
    else z = ug_atan(q);
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return UG_PI - (z - UG_PI_LO);
        default: return (z - UG_PI_LO) - UG_PI;
    }
}

/* ---- asin / acos ---- */
UG_HD double ug__asinR(double t) {
    const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
                 qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
    double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
    return p / q;
}
UG_HD double ug_asin(double x) {
    const double pio4_hi = 7.85398163397448278999e-01;
    double ax = ug_fabs(x), t, w;
    if (ax >= 1.0) {
        if (ax == 1.0) return x * UG_PIO2_HI + x * UG_PIO2_LO;
        return (x - x) / (x - x);
    }
    if (ax < 0.5) {
        if (ax < 3.725290298461914e-09) return x;
        return x + x * ug__asinR(x * x);
    }
    w = 1.0 - ax;
    t = w * 0.5;
    double r = ug__asinR(t);
    double s = ug_sqrt(t);
    if (ax >= 0.975) {
        t = UG_PIO2_HI - (2.0 * (s + s * r) - UG_PIO2_LO);
    } else {
        double f = ug_trunc_lo(s);
        double c = (t - f * f) / (s + f);
        double p = 2.0 * s * r - (UG_PIO2_LO - 2.0 * c);
        double q = pio4_hi - 2.0 * f;
        t = pio4_hi - (p - q);
    }
    return x < 0.0 ? -t : t;
}
UG_HD double ug_acos(double x) {
    double ax = ug_fabs(x);
    if (ax >= 1.0) {
        if (ax == 1.0) return x > 0.0 ? 0.0 : 2.0 * UG_PIO2_HI + 2.0 * UG_PIO2_LO;
        return (x - x) / (x - x);
    }
    if (ax < 0.5) {
        if (ax <= 6.938893903907228e-18) return UG_PIO2_HI + UG_PIO2_LO;
        double r = ug__asinR(x * x);
        return UG_PIO2_HI - (x - (UG_PIO2_LO - x * r));
    }
    if (x < 0.0) {
        double z = (1.0 + x) * 0.5;
        double s = ug_sqrt(z);
        double r = ug__asinR(z);
        double w = r * s - UG_PIO2_LO;
        return UG_PI - 2.0 * (s + w);
    }
    double z = (1.0 - x) * 0.5;
    double s = ug_sqrt(z);
    double df = ug_trunc_lo(s);
    double c = (z - df * df) / (s + df);
    double r = ug__asinR(z);
    double w = r * s + c;
    return 2.0 * (df + w);
}

/* ---- expm1 / tanh (fdlibm s_expm1.c, s_tanh.c) ---- */
UG_HD double ug_expm1(double x) {
    const double o_threshold = 7.09782712893383973096e+02, ln2_hi = 6.93147180369123816490e-01,
                 ln2_lo = 1.90821492927058770002e-10, invln2 = 1.44269504088896338700e+00,
                 Q1 = -3.33333333333331316428e-02, Q2 = 1.58730158725481460165e-03,
                 Q3 = -7.93650757867487942473e-05, Q4 = 4.00821782732936239552e-06,
                 Q5 = -2.01099218183624371326e-07;
    double hi, lo, c = 0.0, t, y, e;
    int k;
    double ax = ug_fabs(x);
    if (ax >= 38.816242111356935) {
        if (x > o_threshold) return 1.0e300 * 1.0e300;
        if (x < 0.0) return -1.0;
    }
    if (ax > 3.4657359027997265e-01) {
        if (ax < 1.0397207708399179) {
            if (x > 0.0) { hi = x - ln2_hi; lo = ln2_lo; k = 1; }
            else { hi = x + ln2_hi; lo = -ln2_lo; k = -1; }
        } else {
            k = (int)ug_rint(invln2 * x);
            t = (double)k;
            hi = x - t * ln2_hi;
            lo = t * ln2_lo;
        }
        x = hi - lo;
        c = (hi - x) - lo;
    } else if (ax < 5.551115123125783e-17) {
        return x;
    } else {
        k = 0;
    }
    double hfx = 0.5 * x;
    double hxs = x * hfx;
    double r1 = 1.0 + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
    t = 3.0 - r1 * hfx;
    e = hxs * ((r1 - t) / (6.0 - x * t));
    if (k == 0) return x - (x * e - hxs);
    e = (x * (e - c) - c);
    e -= hxs;
    if (k == -1) return 0.5 * (x - e) - 0.5;
    if (k == 1) {
        if (x < -0.25) return -2.0 * (e - (x + 0.5));
        return 1.0 + 2.0 * (x - e);
    }
    if (k <= -2 || k > 56) {
        y = 1.0 - (e - x);
        y = ug_scalbn(y, k);
        return y - 1.0;
    }
    if (k < 20) {
        t = 1.0 - ug_scalbn(1.0, -k); /* 1 - 2^-k */
        y = t - (e - x);
        y = ug_scalbn(y, k);
    } else {
        t = ug_scalbn(1.0, -k);
        y = x - (e + t);
        y += 1.0;
        y = ug_scalbn(y, k);
    }
    return y;
}
UG_HD double ug_tanh(double x) {
    double ax = ug_fabs(x), z, t;
    if (ax >= 22.0) z = 1.0;
    else if (ax < 2.7755575615628914e-17) return x;
    else if (ax >= 1.0) { t = ug_expm1(2.0 * ax); z = 1.0 - 2.0 / (t + 2.0); }
    else { t = ug_expm1(-2.0 * ax); z = -t / (t + 2.0); }
    return x < 0.0 ? -z : z;
}

#endif
