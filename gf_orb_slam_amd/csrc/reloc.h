// Track-loss paths of the tracking step (reloc.hip): TrackPreviousFrame and
// Relocalisation, the per-stream state they read and the scratch they use.
// frontend.hip fills a TrackLossArgs once per front end and launches the two
// stages inside its step.
#pragma once
#include "common.h"
#include "match_common.h"

namespace gf {

constexpr int RL_NC = 64;     // relocalisation candidate slots per stream (the keyframe-graph cap)
constexpr int RL_LCAP = 300;  // PnP hypotheses one iterate() call can need (mRansacMaxIts <= 300)
constexpr int RL_WORK = 12;   // doubles per correspondence of the PnP refine buffer (pnp_core.h kWork)

// Frame grid scratch per stream: cell_start [NCELLS + 1], items / scratch /
// claim [cap] each.
__host__ __device__ inline size_t grid_ints(int cap) { return (size_t)NCELLS + 1 + 3 * (size_t)cap; }

// Device view of a keyframe database (gf_kfdb) plus its inverted file.
struct KfdbDev {
    int nkf;
    const int32_t* kp_off;
    const gf_keypoint* kps;
    const uint8_t* desc;
    const int32_t* bow_off;
    const int32_t* bow_words;
    const double* bow_values;
    const int32_t* fv_off;
    const int32_t* fv_nodes;
    const int32_t* fv_start;
    const int32_t* fv_feats;
    // mvInvertedFile: inv_words ascending, keyframes of word w at inv_kf[inv_off[w] .. inv_off[w + 1])
    int nw;
    const int32_t* inv_words;
    const int32_t* inv_off;
    const int32_t* inv_kf;
};

struct TrackLossArgs {
    int B, cap, M, budget, nlevels;
    FrameConst fc;
    float inv_sigma2[16], level_sigma2[16];
    // current frame
    const gf_keypoint* kps;
    const uint8_t* desc;
    const int32_t* nkp;
    int32_t* kp2mp;
    int32_t* score;
    uint8_t* outl;
    float* Tcw;
    // last frame
    const gf_keypoint* last_kps;
    const uint8_t* last_desc;
    const int32_t* last_nkp;
    const int32_t* last_kp2mp;
    const float* last_pos;
    const float* Tcw_last;
    // the stream maps (map indices of kp2mp)
    const gf_map_point* gmap;
    const uint8_t* gdesc;
    // state
    int32_t* track;  // [B][GF_TR_N]
    int32_t* stats;  // [GF_FE_NSTAT][B]
    gf_rng* rng;
    const int32_t* kf_count;  // [B] keyframes of the stream's graph (-1: no graph; assumed > 5)
    const int32_t* gnmp;      // [B] the stream maps' sizes
    // gates of the TrackLocalMap stages (written for every stream)
    int32_t* nkp_tl;    // [B] nkp when TrackLocalMap runs, else 0
    int32_t* nkp_fi;    // [B] nkp when its FRAME_INFO_MATRIX pass runs, else 0
    int32_t* gate_tl;   // [B]
    int32_t* gate_fi;   // [B]
    float* th_m2;       // [B] 5 within 2 frames of a relocalisation, else 1
    int32_t* nmp_step;  // [B] null with keyframe graphs; else gnmp when TrackLocalMap runs, else 0
    // scratch per stream
    int32_t* grid;        // [B][grid_ints(cap)]
    int32_t* rec;         // [B][cap] rotation-histogram records
    gf_pose_edge* edges;  // [B][cap]
    int32_t* edge_kp;     // [B][cap]
    uint8_t* eoutl;       // [B][cap]
    double* pwork;        // [B][3 cap]
    int32_t* pint;        // [B][4] nedges, inliers, iterations
    // relocalisation (kfdb null: no stream has a database)
    const KfdbDev* kfdb;        // [B] (nkf 0: none)
    int rl_on;                  // the step computes candidates (a vocabulary and some database set)
    const gf_covis_map* covis;  // [B] the streams' keyframe graphs (device)
    gf_reloc_kf* rkf;           // [B][RL_NC]
    const int32_t* rl_gate;     // [B] 1: the stream relocalises this step
    const int32_t* words;       // [B][cap] the frame's BowVector
    const double* values;
    const int32_t* nwords;
    const int32_t* fv_nodes;  // [B][cap] its FeatureVector
    const int32_t* fv_start;  // [B][cap + 1]
    const int32_t* fv_feats;  // [B][cap]
    const int32_t* nfv;
    int ncs;                  // candidate slots per stream in pairs / bow_out (max keyframes over the streams)
    BowPairDev* pairs;        // [B][ncs]
    int32_t* bow_out;         // [B][ncs][cap]
    int32_t* bow_nm;          // [B][ncs]
    int32_t* cands;           // [B][RL_NC]
    int32_t* ncand;           // [B]
    gf_pnp_state* pst;        // [B][RL_NC]
    uint8_t* pbest;           // [B][RL_NC][cap]
    float* p3d;               // [B][cap][3]
    float* p2d;               // [B][cap][2]
    float* psig;              // [B][cap]
    int32_t* pidx;            // [B][cap]
    uint8_t* pinl;            // [B][cap]
    int32_t* pdraws;          // [B][RL_LCAP][8]
    double* prt;              // [B][RL_LCAP][12]
    int32_t* pcnt;            // [B][RL_LCAP]
    double* pwk;              // [B][cap][RL_WORK]
    float* ptcw;              // [B][16]
    int32_t* pflags;          // [B][2] flags, inliers of the last iterate()
};

// The device arrays of a keyframe database (gf_kfdb_create).
const KfdbDev& kfdb_dev(const gf_kfdb* db);

// DetectRelocalisationCandidates for the streams that relocalise and their
// SearchByBoW pairs (k_match_bow then runs over A.pairs).
int reloc_candidates(gf_ctx* ctx, const TrackLossArgs& A, hipStream_t s);
// After TrackWithMotionModel: its failure test, TrackPreviousFrame for the
// streams that need it, Relocalisation for the LOST ones; sets GF_TR_OK.
int track_loss(gf_ctx* ctx, const TrackLossArgs& A, hipStream_t s);

}  // namespace gf
