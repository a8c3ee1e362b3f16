// TEST INFRASTRUCTURE: checks the device restatement of glibc's sinf/cosf
// (gf_orb_slam_amd/csrc/libm_sincosf.h, compiled here for the host) against
// the C library itself, float by float.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../gf_orb_slam_amd/csrc/libm_sincosf.h"

extern "C" int orc_libm_sincosf_mismatches(float lo, float hi, long long* nsin, long long* ncos, long long* nchecked) {
    uint32_t a, b;
    memcpy(&a, &lo, 4);
    memcpy(&b, &hi, 4);
    long long ns = 0, nc = 0, n = 0;
    for (uint32_t u = a; u <= b; u++) {
        float x;
        memcpy(&x, &u, 4);
        ns += gflibm::sinf(x) != ::sinf(x);
        nc += gflibm::cosf(x) != ::cosf(x);
        n++;
        if (u == 0xffffffffu) break;
    }
    *nsin = ns;
    *ncos = nc;
    *nchecked = n;
    return 0;
}
