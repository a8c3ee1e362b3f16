// sinf / cosf as glibc >= 2.28 computes them (sysdeps/ieee754/flt-32/s_sinf.c,
// s_cosf.c, sincosf.h, sincosf_data.c — the ARM optimized-routines
// algorithm): the float argument widened to double, reduced by the nearest
// multiple of pi/2 for |y| >= ~pi/4, and a degree-9 odd (sin) or degree-8
// even (cos) polynomial evaluated in double, rounded once to float.
//
// The reference's rBRIEF takes `(float)cos(angle)` of a float under
// `using namespace std` (ORBextractor.cc:75, :167), i.e. glibc's cosf/sinf,
// which are not correctly rounded (about 1 in 1000 arguments of [0, 2pi)
// differ from (float)cos((double)x)). This restatement reproduces them bit
// for bit: tests/test_oracle_extract.py compares it with the C library over
// every float in [0, 2pi] (the range of the keypoint angles), for both the
// FMA and the plain build of glibc (they agree there).
//
// Host and device: plain arithmetic, no contraction (-ffp-contract=off).
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define GF_LIBM_HD __host__ __device__ __forceinline__
#else
#define GF_LIBM_HD inline
#endif

namespace gflibm {

struct SinCosTab {
    double sign[4];
    double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};

GF_LIBM_HD const SinCosTab& sincos_tab(int i) {
    // table [1] is table [0] with the cosine coefficients negated (n & 2)
    static constexpr SinCosTab T[2] = {
        {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
         0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
         0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
        {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
         -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
         0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
    return T[i];
}

GF_LIBM_HD uint32_t abstop12(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return (u >> 20) & 0x7ff;
}

GF_LIBM_HD float sincos_poly(double x, double x2, const SinCosTab& p, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = p.s2 + x2 * p.s3;
        const double x7 = x3 * x2;
        const double s = x + x3 * p.s1;
        return (float)(s + x7 * s1);
    }
    const double x4 = x2 * x2;
    const double c2 = p.c3 + x2 * p.c4;
    const double c1 = p.c0 + x2 * p.c1;
    const double x6 = x4 * x2;
    const double c = c1 + x4 * p.c2;
    return (float)(c + x6 * c2);
}

GF_LIBM_HD double reduce_fast(double x, const SinCosTab& p, int& n) {
    const double r = x * p.hpi_inv;
    n = ((int32_t)r + 0x800000) >> 24;
    return x - n * p.hpi;
}

// |y| < 120 (keypoint angles are in [0, 2pi)); larger arguments take glibc's
// slow reduction, which is not restated: they fall back to the double path.
GF_LIBM_HD float sinf(float y) {
    double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sincos_poly(x, x * x, sincos_tab(0), 0);
    }
    if (abstop12(y) >= abstop12(120.0f)) return (float)::sin(x);
    int n;
    x = reduce_fast(x, sincos_tab(0), n);
    const double s = sincos_tab(0).sign[n & 3];
    return sincos_poly(x * s, x * x, sincos_tab((n & 2) ? 1 : 0), n);
}

GF_LIBM_HD float cosf(float y) {
    double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sincos_poly(x, x * x, sincos_tab(0), 1);
    }
    if (abstop12(y) >= abstop12(120.0f)) return (float)::cos(x);
    int n;
    x = reduce_fast(x, sincos_tab(0), n);
    const double s = sincos_tab(0).sign[n & 3];
    return sincos_poly(x * s, x * x, sincos_tab((n & 2) ? 1 : 0), n ^ 1);
}

}  // namespace gflibm
