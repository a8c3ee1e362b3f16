// glibc random_r (TYPE_3: x[i] = x[i-3] + x[i-31], output >> 1) — the
// generator behind std::srand/std::rand that the reference's lazier greedy
// draws from (Observability.cc:1348, :2895). Host and device share this port.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GFR_HD __host__ __device__ __forceinline__
#else
#define GFR_HD inline
#endif

namespace gfrng {

GFR_HD int32_t next(int32_t* st, int32_t* f, int32_t* r) {
    uint32_t val = (uint32_t)st[*f] + (uint32_t)st[*r];
    st[*f] = (int32_t)val;
    int32_t res = (int32_t)(val >> 1);
    ++*f;
    if (*f >= 31) {
        *f = 0;
        ++*r;
    } else {
        ++*r;
        if (*r >= 31) *r = 0;
    }
    return res;
}

GFR_HD void seed(int32_t* st, int32_t* f, int32_t* r, uint32_t s) {
    if (s == 0) s = 1;
    st[0] = (int32_t)s;
    int32_t word = (int32_t)s;  // glibc keeps `word` as int32_t
    for (int i = 1; i < 31; ++i) {
        long long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        st[i] = word;
    }
    *f = 3;
    *r = 0;
    for (int k = 0; k < 310; k++) (void)next(st, f, r);
}

}  // namespace gfrng
