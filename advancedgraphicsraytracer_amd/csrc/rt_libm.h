// rt_libm.h -- the path's transcendentals as fixed sequences of IEEE double + and *.
//
// Renderer::Trace needs cosf/sinf (ObjectMaterial.h:32-33, the cosine-weighted bounce) and
// expf (Dielectric.h:15-17, Beer's law).  The reference takes them from the platform libm
// (MSVC CRT); their last bit is implementation-defined and cannot be pinned.  Here they are
// evaluated in double with fdlibm's minimax kernels and rounded once to float -- the
// correctly rounded float in all but astronomically rare near-tie cases -- using only basic
// operations, so the gfx950 kernels (built with -ffp-contract=off) and the CPU oracle
// (oracle/rt_oracle.c, same sequence) agree bit for bit without any device libm.
// Cheaper than ocml's general double cos/sin/exp (no Payne-Hanek path, few registers).
#pragma once

#ifndef RT_LIBM_FN
#define RT_LIBM_FN __host__ __device__ __forceinline__
#endif

namespace rt {

// round-to-nearest-even integer of |v| < 2^51 with basic ops only
RT_LIBM_FN double rint_small(double v) {
    const double shifter = 6755399441055744.0;   // 1.5 * 2^52
    return (v + shifter) - shifter;
}

// fdlibm __kernel_sin / __kernel_cos on [-pi/4, pi/4] (tail terms y = 0)
RT_LIBM_FN double ksin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x, v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}
RT_LIBM_FN double kcos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}

// sin and cos of a float angle with |a| < 2^20 (the path only passes 2*pi*[0,1))
RT_LIBM_FN void sincos_f(float a, float &s, float &c) {
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;    // first 33 bits of pi/2
    const double pio2_1t = 6.07710050650619224932e-11;   // pi/2 - pio2_1
    double x = (double)a;
    double k = rint_small(x * invpio2);
    double r = (x - k * pio2_1) - k * pio2_1t;           // k * pio2_1 is exact for |k| < 2^20
    double sr = ksin(r), cr = kcos(r);
    int q = (int)k & 3;
    double sv = q == 0 ? sr : q == 1 ? cr : q == 2 ? -sr : -cr;
    double cv = q == 0 ? cr : q == 1 ? -sr : q == 2 ? -cr : sr;
    s = (float)sv;
    c = (float)cv;
}

// exp of a float, rounded to float (fdlibm __ieee754_exp's reduction and rational kernel)
RT_LIBM_FN float exp_f(float a) {
    if (!(a == a)) return a;
    if (a > 88.8f) return 1.0f / 0.0f;
    if (a < -104.0f) return 0.0f;
    const double ln2hi = 6.93147180369123816490e-01, ln2lo = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    double x = (double)a;
    double k = rint_small(x * invln2);
    double hi = x - k * ln2hi, lo = k * ln2lo;
    double r = hi - lo;
    double t = r * r;
    double cc = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1.0 - ((lo - (r * cc) / (2.0 - cc)) - hi);
    // y * 2^k is exact in double for k in [-151, 129]; one rounding to float at the end
    const unsigned long long bits = (unsigned long long)((long long)k + 1023) << 52;
    return (float)(y * __builtin_bit_cast(double, bits));
}

}  // namespace rt
