// Drives the C++ drop-in layer (include/gfslam/orbslam.h) the way Tracking
// does for one frame, from files written by tests/test_dropin_gpu.py, and
// dumps every result for the test to compare with the CPU oracle.
//   dropin_frontend <dir>
// <dir>/params.txt : w h fx fy cx cy M  then 16 floats Tcw
// <dir>/img.u8     : h*w bytes
// <dir>/map.bin    : M x (gf_map_point 32 B + descriptor 32 B)
// <dir>/voc.bin    : a DBoW2 binary vocabulary
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "gfslam/orbslam.h"

using namespace ORB_SLAM;

template <typename T>
static void dump(const std::string& path, const T* p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), sizeof(T) * n);
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string dir = argv[1];
    int w, h, M;
    float K[4], T0[16];
    {
        std::ifstream p(dir + "/params.txt");
        p >> w >> h >> K[0] >> K[1] >> K[2] >> K[3] >> M;
        for (float& t : T0) p >> t;
    }
    std::vector<uint8_t> img((size_t)w * h);
    std::ifstream(dir + "/img.u8", std::ios::binary).read(reinterpret_cast<char*>(img.data()), img.size());
    std::vector<MapPoint> mps(M);
    {
        std::ifstream f(dir + "/map.bin", std::ios::binary);
        for (int i = 0; i < M; i++) {
            gf_map_point g;
            f.read(reinterpret_cast<char*>(&g), sizeof(g));
            f.read(reinterpret_cast<char*>(mps[i].mDescriptor), 32);
            for (int k = 0; k < 3; k++) {
                mps[i].mWorldPos[k] = g.pos[k];
                mps[i].mNormalVector[k] = g.normal[k];
            }
            mps[i].mfMinDistance = g.min_dist;
            mps[i].mfMaxDistance = g.max_dist;
        }
    }
    std::vector<MapPoint*> local(M);
    for (int i = 0; i < M; i++) local[i] = &mps[i];

    try {
        // Frame::Frame -> ORBextractor (E1-E8)
        ORBextractor extractor(1000, 1.2f, 8, ORBextractor::FAST_SCORE, 20);
        ImageView im{img.data(), w, h, (size_t)w};
        Frame F(im, 0.0, &extractor, K);
        dump(dir + "/kps.bin", F.mvKeys.data(), F.N);
        dump(dir + "/desc.bin", F.mDescriptors.data.data(), F.mDescriptors.data.size());

        // SearchLocalPoints: isInFrustum (M7) + SearchByProjection(F, local, 1) (M2)
        F.SetPose(T0);
        const int nview = F.isInFrustum(local, 0.5f);
        ORBmatcher matcher(0.8f);
        const int nm = matcher.SearchByProjection(F, local, 1.0f);
        std::vector<int32_t> kp2mp(F.N);
        for (int i = 0; i < F.N; i++) kp2mp[i] = F.mvpMapPoints[i] ? (int32_t)(F.mvpMapPoints[i] - mps.data()) : -1;
        dump(dir + "/kp2mp_m2.i32", kp2mp.data(), F.N);

        // PoseOptimization (P1-P4)
        const int ninl = Optimizer::PoseOptimization(&F);
        dump(dir + "/pose.f32", F.mTcw, 16);
        std::vector<uint8_t> outl(F.N);
        for (int i = 0; i < F.N; i++) outl[i] = F.mvbOutlier[i];
        dump(dir + "/outl.u8", outl.data(), F.N);

        // SearchByProjection(Cur, Last, 15) (M3): the same image as the next frame
        Frame F2(im, 0.05, &extractor, K);
        F2.SetPose(F.mTcw);
        ORBmatcher m3(0.9f, true);
        const int n3 = m3.SearchByProjection(F2, F, 15.0f);
        std::vector<int32_t> kp2mp3(F2.N);
        for (int i = 0; i < F2.N; i++)
            kp2mp3[i] = F2.mvpMapPoints[i] ? (int32_t)(F2.mvpMapPoints[i] - mps.data()) : -1;
        dump(dir + "/kp2mp_m3.i32", kp2mp3.data(), F2.N);

        // GF: kinematics + MAP_INFO_MATRIX + active matching (G1-G7)
        Observability obs(K[0], K[1], h, w, K[2], K[3], 0, 0);
        obs.mBoundXInFrame = (int)(0.1 * w);
        obs.mBoundYInFrame = (int)(0.1 * h);
        float Twc[16];
        F2.getTwc(Twc);
        obs.updatePWLSVec(0.0, F.mTcw, 0.05, Twc);
        obs.predictPWLSVec(0.05, 1);
        obs.mKineIdx = 0;
        obs.mnFrameId = F2.mnId;
        obs.pFrame = &F2;
        for (int i = 0; i < F2.N; i++) {
            if (F2.mvpMapPoints[i]) F2.mvpMapPoints[i]->mbTrackInView = false;
        }
        std::vector<MapPoint*> rest;
        for (MapPoint* p : local) {
            bool matched = false;
            for (MapPoint* q : F2.mvpMapPoints) matched |= q == p;
            if (!matched) rest.push_back(p);
        }
        F2.isInFrustum(rest, 0.5f);
        obs.mMapPoints = &local;
        obs.runMatrixBuilding(MAP_INFO_MATRIX, 1.0, true, false);
        double base[49] = {};
        for (int i = 0; i < 7; i++) base[8 * i] = 1e-5;
        obs.srand(5);
        const int nact = obs.runActiveMapMatching(&F2, FRAME_INFO_MATRIX, base, 1.0f, matcher, 40, 1.0);
        std::vector<int32_t> kp2mp_a(F2.N);
        for (int i = 0; i < F2.N; i++)
            kp2mp_a[i] = F2.mvpMapPoints[i] ? (int32_t)(F2.mvpMapPoints[i] - mps.data()) : -1;
        dump(dir + "/kp2mp_act.i32", kp2mp_a.data(), F2.N);
        std::vector<double> Xv(obs.kinematic[0].Xv, obs.kinematic[0].Xv + 13);
        dump(dir + "/xv.f64", Xv.data(), 13);

        FILE* s = std::fopen((dir + "/summary.txt").c_str(), "w");
        std::fprintf(s, "%d %d %d %d %d %d %d %d\n", F.N, nview, nm, ninl, F2.N, n3, nact,
                     ORBmatcher::DescriptorDistance(F.mDescriptors.ptr(0), F.mDescriptors.ptr(1)));
        std::fclose(s);

        auto idx_of = [&](const std::vector<MapPoint*>& v) {
            std::vector<int32_t> o(v.size());
            for (size_t i = 0; i < v.size(); i++) o[i] = v[i] ? (int32_t)(v[i] - mps.data()) : -1;
            return o;
        };

        // Frame::ComputeBoW (D1) and SearchByBoW KeyFrame-Frame / KeyFrame-KeyFrame (M6)
        ORBVocabulary voc;
        if (!voc.loadFromBinaryFile(dir + "/voc.bin") || voc.loadFromTextFile(dir + "/voc.bin")) return 3;
        F.mpORBvocabulary = &voc;
        F.ComputeBoW();
        F2.mpORBvocabulary = &voc;
        F2.ComputeBoW();
        dump(dir + "/bow_words.i32", F.mBowVec.words.data(), F.mBowVec.words.size());
        dump(dir + "/bow_values.f64", F.mBowVec.values.data(), F.mBowVec.values.size());
        dump(dir + "/fv_nodes.i32", F.mFeatVec.nodes.data(), F.mFeatVec.nodes.size());
        dump(dir + "/fv_start.i32", F.mFeatVec.start.data(), F.mFeatVec.start.size());
        dump(dir + "/fv_feats.i32", F.mFeatVec.feats.data(), F.mFeatVec.feats.size());
        KeyFrame KF(F);    // map points of F: the M2 claims
        KeyFrame KF2(F2);  // map points of F2: M3 + active matching
        ORBmatcher mbow(0.75f, true);
        std::vector<MapPoint*> vm, v12;
        const int nb0 = mbow.SearchByBoW(&KF, F2, vm);
        const int nb1 = mbow.SearchByBoW(&KF, &KF2, v12);
        dump(dir + "/bow_kf_f.i32", idx_of(vm).data(), vm.size());
        dump(dir + "/bow_kf_kf.i32", idx_of(v12).data(), v12.size());

        // SearchByProjection_OnePoint (M4) then SearchByProjection_Budget (M5) on a fresh frame
        Frame F3(im, 0.1, &extractor, K);
        F3.SetPose(F.mTcw);
        F3.isInFrustum(local, 0.5f);
        MapPoint* p0 = nullptr;
        for (MapPoint* q : F.mvpMapPoints)
            if (q) {
                p0 = q;
                break;
            }
        ORBmatcher m8(0.8f);
        const int one = m8.SearchByProjection_OnePoint(F3, p0, 1.0f);
        const int nbud0 = m8.SearchByProjection_Budget(F3, local, 0.8f, 0.0);  // no time: nothing
        const int nbud = m8.SearchByProjection_Budget(F3, local, 0.8f, 1.0);
        dump(dir + "/budget_kp2mp.i32", idx_of(F3.mvpMapPoints).data(), F3.N);
        dump(dir + "/budget_score.i32", F3.mvpMatchScore.data(), F3.N);
        long found = 0;
        for (const MapPoint& q : mps) found += q.mnFound - 1;

        // Observability::setSelction_Number over the local map (G7, map scale)
        Observability sel(K[0], K[1], h, w, K[2], K[3], 0, 0);
        sel.mBoundXInFrame = (int)(0.1 * w);
        sel.mBoundYInFrame = (int)(0.1 * h);
        sel.updatePWLSVec(0.0, F.mTcw, 0.05, Twc);
        sel.predictPWLSVec(0.05, 2);
        sel.mNumThreads = 8;
        sel.srand(9);
        std::vector<GoodPoint> good;
        const bool no_time = sel.setSelction_Number(300, 3, 0.0, &local, &good);
        // points updated this frame before the selection (FRAME_INFO_MATRIX of
        // matched points: their own block and score) keep them: every 7th
        // local point with a scaled identity block and score 0.5, every 11th
        // with ObsScore -1 (no pool entry)
        sel.mnFrameId = 5;
        for (size_t i = 0; i < local.size(); i++) {
            MapPoint* q = local[i];
            if (i % 7 == 3) {
                q->updateAtFrameId = 5;
                for (int e = 0; e < 49; e++) q->ObsMat[e] = (e % 8 == 0) ? 1e3 * (1 + (double)(i % 5)) : 0.0;
                q->hasObsMat = true;
                q->ObsScore = 0.5;
            } else if (i % 11 == 4) {
                q->updateAtFrameId = 5;
                q->ObsScore = -1.0;
            }
        }
        const bool ok = sel.setSelction_Number(300, 3, 1.0, &local, &good);
        std::vector<double> lscore;
        std::vector<int32_t> lstamp;
        for (MapPoint* q : local) {
            lscore.push_back(q->ObsScore);
            lstamp.push_back((int32_t)q->updateAtFrameId);
        }
        dump(dir + "/select_scores.f64", lscore.data(), lscore.size());
        dump(dir + "/select_stamps.i32", lstamp.data(), lstamp.size());
        std::vector<int32_t> gidx;
        for (const GoodPoint& g : good) gidx.push_back((int32_t)g.idx);
        dump(dir + "/select.i32", gidx.data(), gidx.size());
        std::vector<double> gblk;
        for (const GoodPoint& g : good) gblk.insert(gblk.end(), g.obs_block.begin(), g.obs_block.end());
        dump(dir + "/select_blocks.f64", gblk.data(), gblk.size());

        FILE* s2 = std::fopen((dir + "/summary2.txt").c_str(), "w");
        std::fprintf(s2, "%d %d %d %d %d %ld %d %d %d\n", nb0, nb1, (int)(p0 ? p0 - mps.data() : -1), one, nbud0,
                     found, nbud, (int)no_time, (int)ok);
        std::fclose(s2);
    } catch (const GpuError& e) {
        std::fprintf(stderr, "GpuError %d: %s\n", e.code, e.what());
        return 1;
    }
    return 0;
}
