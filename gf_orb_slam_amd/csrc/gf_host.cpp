// Host-side pieces of the good-feature module that the reference runs as
// scalar per-frame state updates ("stays on host"):
// glibc rand() state (std::srand/std::rand port) and the constant-velocity
// PWLS kinematics of Observability::updatePWLSVec / predictPWLSVec
// (include/Observability.h:222-295, include/Util.hpp:787-1005).
#include <math.h>
#include <string.h>

#include <cfloat>
#include <cmath>

#include "../../include/gfslam/abi.h"
#include "kine.h"
#include "rng.h"

using namespace gfkine;


extern "C" {

int gf_rng_seed(gf_rng* rng, uint32_t seed) {
    if (!rng) return GF_ERR_ARG;
    gfrng::seed(rng->state, &rng->f, &rng->r, seed);
    return GF_OK;
}

int gf_rng_next(gf_rng* rng, int32_t* out, int n) {
    if (!rng || (n > 0 && !out)) return GF_ERR_ARG;
    for (int i = 0; i < n; i++) out[i] = gfrng::next(rng->state, &rng->f, &rng->r);
    return GF_OK;
}

int gf_obs_update(double t_prev, const float* Tcw_prev, double t_cur, const float* Twc_cur, double* Xv) {
    if (!Tcw_prev || !Twc_cur || !Xv) return GF_ERR_ARG;
    gfkine::obs_update(t_prev, Tcw_prev, t_cur, Twc_cur, Xv);
    return GF_OK;
}

int gf_obs_predict(const double* Xv, double dt, int nseg, gf_kine* out) {
    if (!Xv || !out || nseg < 0) return GF_ERR_ARG;
    double cur[13];
    memcpy(cur, Xv, sizeof(cur));
    for (int s = 0; s < nseg; s++) {
        gf_kine& K = out[s];
        K.dt = (float)dt;  // KineStruct.dt = float(dt)
        K.dt_inseg = (float)K.dt / (float)13;
        memcpy(K.Xv, cur, sizeof(cur));
        state_to_Tcw(K.Xv, K.Tcw);
        f_blocks(K.Xv, K.dt_inseg, K.F_Q_inSeg, K.F_Omg_inSeg);
        f_blocks(K.Xv, K.dt, K.F_Q, K.F_Omg);
        double nxt[13];
        propagate_state(K.Xv, K.dt, nxt);
        memcpy(cur, nxt, sizeof(cur));
    }
    return GF_OK;
}

}  // extern "C"
