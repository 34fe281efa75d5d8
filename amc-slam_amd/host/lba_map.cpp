// lba_map.cpp — map classes of lba_map.hpp and the window-snapshot reader / writer.
//
// Each method cites the reference function it restates.  Float arithmetic follows Sophus'
// formulas (quaternion product, q v q*, normalise on construction), summed in plain order.
#include "lba_map.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <type_traits>

#include "../../include/amc_lba_map.h"
#include "../csrc/lba_math.hpp"

namespace amc_slam {

// ------------------------------------------------------------------ SE3 (Sophus, float)
template <typename T>
static void qnorm(T* q) {   // so3.hpp:297-303
    const T n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; ++i) q[i] /= n;
}

template <typename T>
static void qrotate(const T* q, const T* p, T* o) {   // so3.hpp:363-366: p + w uv + v x uv, uv = 2 v x p
    T uv[3] = {q[1] * p[2] - q[2] * p[1], q[2] * p[0] - q[0] * p[2], q[0] * p[1] - q[1] * p[0]};
    for (int i = 0; i < 3; ++i) uv[i] += uv[i];
    const T c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    for (int i = 0; i < 3; ++i) o[i] = p[i] + q[3] * uv[i] + c[i];
}

template <typename T>
static void qproduct(const T* a, const T* b, T* o) {   // so3.hpp:325-339 (x, y, z, w storage)
    const T w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    const T x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    const T y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    const T z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z; o[3] = w;
    qnorm(o);
}

template <typename S>
static S se3_inverse(const S& a) {   // se3.hpp:208-211
    S r;
    r.q[0] = -a.q[0]; r.q[1] = -a.q[1]; r.q[2] = -a.q[2]; r.q[3] = a.q[3];
    qnorm(r.q);
    std::remove_cv_t<std::remove_reference_t<decltype(a.t[0])>> mt[3] = {-a.t[0], -a.t[1], -a.t[2]};
    qrotate(r.q, mt, r.t);
    return r;
}

SE3f SE3f::inverse() const { return se3_inverse(*this); }

SE3f SE3f::operator*(const SE3f& o) const {   // se3.hpp:304-308
    SE3f r;
    qproduct(q, o.q, r.q);
    float rt[3];
    qrotate(q, o.t, rt);
    for (int i = 0; i < 3; ++i) r.t[i] = t[i] + rt[i];
    return r;
}

Vec3f SE3f::act(const Vec3f& p) const {
    const float pi[3] = {p.x, p.y, p.z};
    float o[3];
    qrotate(q, pi, o);
    return Vec3f{o[0] + t[0], o[1] + t[1], o[2] + t[2]};
}

SE3d SE3d::inverse() const { return se3_inverse(*this); }

SE3f SE3d::cast_float() const {
    SE3f f;
    for (int i = 0; i < 4; ++i) f.q[i] = (float)q[i];
    qnorm(f.q);
    for (int i = 0; i < 3; ++i) f.t[i] = (float)t[i];
    return f;
}

SE3d SE3d::from_float(const SE3f& f) {
    SE3d d;
    for (int i = 0; i < 4; ++i) d.q[i] = (double)f.q[i];
    qnorm(d.q);
    for (int i = 0; i < 3; ++i) d.t[i] = (double)f.t[i];
    return d;
}

bool KFLess::operator()(const MultiKeyFrame* a, const MultiKeyFrame* b) const { return a->mnId < b->mnId; }

// ------------------------------------------------------------------ MultiKeyFrame
// MultiKeyFrame::SetPose(const Sophus::SE3f& Tbw) (src/KeyFrame.cc:116-145): the reference
// camera from Tbc, the asynchronous cameras from the GP query between mPrevKF and this KF at
// their time stamps (GaussianProcess::QueryPose, src/GaussianProcess.cc:5-21).
void MultiKeyFrame::SetPose(const SE3f& Tbw) {
    mTcw = Tbw;
    mTwc = Tbw.inverse();
    const std::vector<CameraParams>& cams = *mvpCamera;
    mvTwc.assign(nCamera, SE3f());
    mvTwc[nCamera - 1] = (cams[nCamera - 1].Tbc.inverse() * mTcw).inverse();
    if (mnId == 0 || !mPrevKF) return;
    const SE3d prevTwb = SE3d::from_float(mPrevKF->GetPose().inverse());
    const SE3d Twb = SE3d::from_float(mTwc);
    lba::SE3 Ta, Tb;
    Ta.q = lba::Quat{prevTwb.q[0], prevTwb.q[1], prevTwb.q[2], prevTwb.q[3]};
    Tb.q = lba::Quat{Twb.q[0], Twb.q[1], Twb.q[2], Twb.q[3]};
    double va[6], vb[6];
    for (int i = 0; i < 3; ++i) { Ta.t[i] = prevTwb.t[i]; Tb.t[i] = Twb.t[i]; }
    for (int i = 0; i < 6; ++i) { va[i] = mPrevKF->GetVelocity()[i]; vb[i] = mVel[i]; }
    lba::GPPair P;
    lba::gp_pair_build(Ta, va, Tb, vb, mPrevKF->mTimeStamp, mTimeStamp, &P, false);
    for (int c = 0; c < nCamera - 1; ++c) {
        // QueryPose: T1 * exp(p2 v1 + l1 xi12 + l2 Jr^-1(xi12) v2), cast to float
        const lba::GPScalars g = lba::gp_scalars(P.t1, P.t2, mvTimeStamps[c]);
        double xi[6];
        for (int i = 0; i < 6; ++i) xi[i] = g.p2 * P.v1[i] + g.l1 * P.xi12[i] + g.l2 * P.w2[i];
        const lba::SE3 T = lba::se3_mul(Ta, lba::se3_exp(xi));
        SE3d Tc;
        Tc.q[0] = T.q.x; Tc.q[1] = T.q.y; Tc.q[2] = T.q.z; Tc.q[3] = T.q.w;
        for (int i = 0; i < 3; ++i) Tc.t[i] = T.t[i];
        mvTwc[c] = Tc.cast_float() * cams[c].Tbc;
    }
}

void MultiKeyFrame::SetCachedPoses(const SE3f& Tbw, const std::vector<SE3f>& Twc) {
    mTcw = Tbw;
    mTwc = Tbw.inverse();
    mvTwc = Twc;
}

void MultiKeyFrame::SetVelocity(const float* v) { std::memcpy(mVel, v, sizeof(mVel)); }

Vec3f MultiKeyFrame::GetCameraCenter(int c) const {
    const SE3f& T = mvTwc[c];
    return Vec3f{T.t[0], T.t[1], T.t[2]};
}

void MultiKeyFrame::EraseMapPointMatch(int idx) { mvpMapPoints[idx] = nullptr; }

void MultiKeyFrame::EraseMapPointMatch(MapPoint* pMP, int cam) {
    const int index = pMP->GetIndexInKeyFrame(this)[cam];
    if (index != -1) mvpMapPoints[index] = nullptr;
}

// ------------------------------------------------------------------ MapPoint
std::vector<int> MapPoint::GetIndexInKeyFrame(MultiKeyFrame* pKF) const {
    auto it = mObservations.find(pKF);
    if (it == mObservations.end()) return std::vector<int>(nCamera, -1);
    return it->second;
}

void MapPoint::AddObservation(MultiKeyFrame* pKF, int idx) {   // src/MapPoint.cc:196-229
    std::vector<int> indexes = mObservations.count(pKF) ? mObservations[pKF] : std::vector<int>(nCamera, -1);
    const int cam = pKF->mmpKeyToCam[idx];
    indexes[cam] = idx;
    mObservations[pKF] = indexes;
    if (cam == nCamera - 1 && pKF->mvuRight[idx] >= 0)
        nObs += 2;
    else
        nObs++;
}

void MapPoint::EraseObservation(MultiKeyFrame* pKF, int c) {   // src/MapPoint.cc:275-315
    bool bBad = false;
    auto it = mObservations.find(pKF);
    if (it != mObservations.end()) {
        std::vector<int> indexes = it->second;
        if (indexes[c] != -1) {
            nObs--;
            if (c == nCamera - 1 && pKF->mvuRight[indexes[c]] >= 0) nObs--;
            indexes[c] = -1;
        }
        bool nobs = true;
        for (int cam = 0; cam < (int)indexes.size(); ++cam)
            if (indexes[cam] != -1) { nobs = false; break; }
        if (nobs) {
            mObservations.erase(it);
            if (mpRefKF == pKF) mpRefKF = mObservations.empty() ? nullptr : mObservations.begin()->first;
        } else {
            it->second = indexes;
        }
        if (nObs <= 2) bBad = true;
    }
    if (bBad) SetBadFlag();
}

void MapPoint::AddGPObservation(MultiKeyFrame* pKF, const GPObs& o) { mObservationsForGPBA.emplace(pKF, o); }

void MapPoint::EraseGPObservation(MultiKeyFrame* pKF, const GPObs& o) {   // src/MapPoint.cc:323-337
    auto range = mObservationsForGPBA.equal_range(pKF);
    for (auto it = range.first; it != range.second; ++it)
        if (it->second == o) { mObservationsForGPBA.erase(it); break; }
}

void MapPoint::SetBadFlag() {   // src/MapPoint.cc:356-386
    auto obs = std::move(mObservations);
    mbBad = true;
    mObservations.clear();
    for (auto& kv : obs)
        for (int i : kv.second)
            if (i != -1) kv.first->EraseMapPointMatch(i);
    mpMap->EraseMapPoint(this);
}

void MapPoint::UpdateNormalAndDepth() {   // src/MapPoint.cc:611-686
    if (mbBad) return;
    const auto& observations = mObservations;   // (the reference copies it under the point's mutex; read in place)
    MultiKeyFrame* pRefKF = mpRefKF;
    const Vec3f Pos = mWorldPos;
    if (observations.empty()) return;
    Vec3f normal;
    int n = 0;
    for (const auto& kv : observations) {
        for (int c = 0; c < nCamera; ++c) {
            if (kv.second[c] != -1) {
                const Vec3f O = kv.first->GetCameraCenter(c);
                const float d[3] = {Pos.x - O.x, Pos.y - O.y, Pos.z - O.z};
                const float nr = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                normal.x = normal.x + d[0] / nr;
                normal.y = normal.y + d[1] / nr;
                normal.z = normal.z + d[2] / nr;
                n++;
            }
        }
    }
    float maxDist = std::numeric_limits<float>::min(), minDist = std::numeric_limits<float>::max();
    auto rit = pRefKF ? observations.find(pRefKF) : observations.end();
    if (rit != observations.end()) {
        const int nLevels = pRefKF->mnScaleLevels;
        const std::vector<float>& sf = *pRefKF->mvScaleFactors;
        for (int c = 0; c < nCamera; ++c) {
            if (rit->second[c] != -1) {
                const Vec3f O = pRefKF->GetCameraCenter(c);
                const float d[3] = {Pos.x - O.x, Pos.y - O.y, Pos.z - O.z};
                const float dist = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                const int level = pRefKF->mvKeysUn[rit->second[c]].octave;
                const float levelScaleFactor = sf[level];
                maxDist = std::max(maxDist, dist * levelScaleFactor);
                minDist = std::min(minDist, dist * levelScaleFactor / sf[nLevels - 1]);
            }
        }
    }
    mfMaxDistance = maxDist;
    mfMinDistance = minDist;
    mNormalVector = Vec3f{normal.x / n, normal.y / n, normal.z / n};
}

// ------------------------------------------------------------------ Map
long unsigned Map::KeyFramesInMap() const {
    long unsigned n = 0;
    for (const auto& k : mvKeyFrames)
        if (!k->mbBad && k->mMapId == mMapId) ++n;
    return n;
}

std::vector<MultiKeyFrame*> Map::GetAllKeyFrames() const {
    std::vector<MultiKeyFrame*> v;
    for (const auto& k : mvKeyFrames)
        if (!k->mbBad && k->mMapId == mMapId) v.push_back(k.get());
    std::stable_sort(v.begin(), v.end(), [](const MultiKeyFrame* a, const MultiKeyFrame* b) { return a->mnId < b->mnId; });
    return v;
}

std::vector<MapPoint*> Map::GetAllMapPoints() const {
    std::vector<MapPoint*> v;
    for (const auto& p : mvMapPoints)
        if (!p->mbBad) v.push_back(p.get());
    std::stable_sort(v.begin(), v.end(), [](const MapPoint* a, const MapPoint* b) { return a->mnId < b->mnId; });
    return v;
}

unsigned long Map::GetInitKFid() const {
    bool any = false;
    unsigned long id = 0;
    for (const auto& k : mvKeyFrames)
        if (k->mMapId == mMapId && (!any || k->mnId < id)) {
            id = k->mnId;
            any = true;
        }
    return id;
}

MultiKeyFrame* Map::kf_by_id(int64_t id) const {
    auto it = mKFById.find(id);
    return it == mKFById.end() ? nullptr : it->second;
}

MapPoint* Map::mp_by_id(int64_t id) const {
    auto it = mMPById.find(id);
    return it == mMPById.end() ? nullptr : it->second;
}

// ------------------------------------------------------------------ snapshot I/O
namespace {

struct Reader {
    const uint8_t* p;
    size_t n, off = 0;
    template <typename T>
    const T* take(int64_t count) {
        const size_t bytes = sizeof(T) * (size_t)count;
        if (count < 0 || off + bytes > n) return nullptr;
        const T* r = reinterpret_cast<const T*>(p + off);
        off += (bytes + 7) & ~size_t(7);
        return r;
    }
};

size_t pad8(size_t b) { return (b + 7) & ~size_t(7); }

}  // namespace

std::unique_ptr<Map> Map::load(const void* bytes, size_t n, std::string* err) {
    Reader rd{static_cast<const uint8_t*>(bytes), n};
    const lbamap_header* h = rd.take<lbamap_header>(1);
    auto fail = [&](const char* m) { if (err) *err = m; return std::unique_ptr<Map>(); };
    if (!h || std::memcmp(h->magic, "AMCSNAP", 8) != 0) return fail("bad snapshot magic");
    if (h->version != LBAMAP_VERSION) return fail("unsupported snapshot version");
    if (h->n_cam < 1 || h->n_cam > LBAMAP_MAX_CAM || h->n_levels < 1 || h->n_levels > LBAMAP_MAX_LEVEL)
        return fail("n_cam / n_levels out of range");
    const lbamap_cam* cams = rd.take<lbamap_cam>(h->n_cam);
    const lbamap_kf* kfs = rd.take<lbamap_kf>(h->n_kf);
    const lbamap_kp* kps = rd.take<lbamap_kp>(h->n_kp);
    const int64_t* cov = rd.take<int64_t>(h->n_covis);
    const lbamap_mp* mps = rd.take<lbamap_mp>(h->n_mp);
    const lbamap_mpobs* mo = rd.take<lbamap_mpobs>(h->n_mpobs);
    const lbamap_gpobs* go = rd.take<lbamap_gpobs>(h->n_gpobs);
    if (!cams || !kfs || !kps || !cov || !mps || !mo || !go) return fail("snapshot truncated");

    auto M = std::make_unique<Map>();
    M->nCamera = h->n_cam;
    std::memcpy(M->mQc, h->qc, sizeof(M->mQc));
    M->mvInvLevelSigma2.assign(h->inv_level_sigma2, h->inv_level_sigma2 + h->n_levels);
    M->mvScaleFactors.assign(h->scale_factor, h->scale_factor + h->n_levels);
    for (int c = 0; c < h->n_cam; ++c) {
        CameraParams cp;
        cp.fx = cams[c].fx; cp.fy = cams[c].fy; cp.cx = cams[c].cx; cp.cy = cams[c].cy;
        std::memcpy(cp.Tbc.q, cams[c].q, sizeof(cp.Tbc.q));
        std::memcpy(cp.Tbc.t, cams[c].t, sizeof(cp.Tbc.t));
        std::memcpy(cp.Rbc_ini, cams[c].rbc_ini, sizeof(cp.Rbc_ini));
        M->mCameras.push_back(cp);
    }
    for (int i = 0; i < h->n_kf; ++i) {
        const lbamap_kf& r = kfs[i];
        auto K = std::make_unique<MultiKeyFrame>();
        K->mnId = (unsigned long)r.id;
        K->mTimeStamp = r.time;
        K->mvTimeStamps.assign(r.cam_time, r.cam_time + h->n_cam);
        K->nCamera = h->n_cam;
        K->mbf = r.bf;
        K->mbBad = r.bad != 0;
        K->mMapId = r.map_id;
        K->mpMap = M.get();
        K->mvInvLevelSigma2 = &M->mvInvLevelSigma2;
        K->mvScaleFactors = &M->mvScaleFactors;
        K->mnScaleLevels = h->n_levels;
        K->mvpCamera = &M->mCameras;
        K->SetVelocity(r.vel);
        if (r.kp_off < 0 || r.n_kp < 0 || (int64_t)r.kp_off + r.n_kp > h->n_kp) return fail("keypoint range");
        for (int j = 0; j < r.n_kp; ++j) {
            const lbamap_kp& kp = kps[r.kp_off + j];
            if (kp.cam < 0 || kp.cam >= h->n_cam || kp.octave < 0 || kp.octave >= h->n_levels)
                return fail("keypoint camera / octave out of range");
            K->mvKeysUn.push_back(KeyPoint{kp.x, kp.y, kp.octave});
            K->mmpKeyToCam.push_back(kp.cam);
            K->mvuRight.push_back(kp.ur);
        }
        if (M->mKFById.count(r.id)) return fail("duplicate keyframe id");
        M->mKFById[r.id] = K.get();
        M->mnMaxKFid = std::max(M->mnMaxKFid, (unsigned long)r.id);
        M->mvKeyFrames.push_back(std::move(K));
    }
    for (int i = 0; i < h->n_kf; ++i) {
        const lbamap_kf& r = kfs[i];
        MultiKeyFrame* K = M->mvKeyFrames[i].get();
        if (r.prev_id >= 0 && !(K->mPrevKF = M->kf_by_id(r.prev_id))) return fail("unknown prev_id");
        if (r.next_id >= 0 && !(K->mNextKF = M->kf_by_id(r.next_id))) return fail("unknown next_id");
        if (r.covis_off < 0 || r.n_covis < 0 || (int64_t)r.covis_off + r.n_covis > h->n_covis) return fail("covis range");
        for (int j = 0; j < r.n_covis; ++j) {
            MultiKeyFrame* C = M->kf_by_id(cov[r.covis_off + j]);
            if (!C) return fail("unknown covisible keyframe");
            K->mvpOrderedConnectedKeyFrames.push_back(C);
        }
    }
    // poses after the links exist: SetPose queries the GP against mPrevKF's pose, so every pose is
    // stored first and the camera poses are derived in a second pass (any snapshot order works)
    for (int pass = 0; pass < 2; ++pass)
        for (int i = 0; i < h->n_kf; ++i) {
            SE3f T;
            std::memcpy(T.q, kfs[i].q, sizeof(T.q));
            std::memcpy(T.t, kfs[i].t, sizeof(T.t));
            if (kfs[i].has_twc) {
                std::vector<SE3f> twc(h->n_cam);
                for (int c = 0; c < h->n_cam; ++c) {
                    std::memcpy(twc[c].q, kfs[i].twc_q[c], sizeof(twc[c].q));
                    std::memcpy(twc[c].t, kfs[i].twc_t[c], sizeof(twc[c].t));
                }
                M->mvKeyFrames[i]->SetCachedPoses(T, twc);
            } else {
                M->mvKeyFrames[i]->SetPose(T);
            }
        }
    for (int i = 0; i < h->n_mp; ++i) {
        const lbamap_mp& r = mps[i];
        auto P = std::make_unique<MapPoint>();
        P->mnId = (unsigned long)r.id;
        P->nCamera = h->n_cam;
        P->mpMap = M.get();
        P->mbBad = r.bad != 0;
        P->mWorldPos = Vec3f{r.pos[0], r.pos[1], r.pos[2]};
        P->mNormalVector = Vec3f{r.normal[0], r.normal[1], r.normal[2]};
        P->mfMinDistance = r.min_dist;
        P->mfMaxDistance = r.max_dist;
        P->mvTrackDepth.assign(r.track_depth, r.track_depth + h->n_cam);
        if (M->mMPById.count(r.id)) return fail("duplicate map point id");
        M->mMPById[r.id] = P.get();
        M->mvMapPoints.push_back(std::move(P));
    }
    for (int i = 0; i < h->n_mp; ++i) {
        const lbamap_mp& r = mps[i];
        MapPoint* P = M->mvMapPoints[i].get();
        P->mpRefKF = r.ref_kf >= 0 ? M->kf_by_id(r.ref_kf) : nullptr;
        if (r.obs_off < 0 || r.n_obs < 0 || (int64_t)r.obs_off + r.n_obs > h->n_mpobs) return fail("obs range");
        if (r.gp_off < 0 || r.n_gp < 0 || (int64_t)r.gp_off + r.n_gp > h->n_gpobs) return fail("gp obs range");
        for (int j = 0; j < r.n_obs; ++j) {
            const lbamap_mpobs& o = mo[r.obs_off + j];
            MultiKeyFrame* K = M->kf_by_id(o.kf_id);
            if (!K) return fail("observation of unknown keyframe");
            for (int c = 0; c < h->n_cam; ++c) {
                const int idx = o.idx[c];
                if (idx < 0) continue;
                if (idx >= (int)K->mvKeysUn.size() || K->mmpKeyToCam[idx] != c) return fail("observation index");
                P->AddObservation(K, idx);
            }
        }
        for (int j = 0; j < r.n_gp; ++j) {
            const lbamap_gpobs& g = go[r.gp_off + j];
            MultiKeyFrame* K = M->kf_by_id(g.kf_id);
            if (!K || g.cam < 0 || g.cam >= h->n_cam || g.octave < 0 || g.octave >= h->n_levels)
                return fail("GP observation");
            GPObs ob;
            ob.time = g.time; ob.cam = g.cam; ob.obs = KeyPoint{g.x, g.y, g.octave}; ob.ur = g.ur;
            P->AddGPObservation(K, ob);
        }
    }
    // keypoint -> map point matches (mvpMapPoints)
    for (int i = 0; i < h->n_kf; ++i) {
        MultiKeyFrame* K = M->mvKeyFrames[i].get();
        K->mvpMapPoints.assign(K->mvKeysUn.size(), nullptr);
        for (int j = 0; j < kfs[i].n_kp; ++j) {
            const int64_t id = kps[kfs[i].kp_off + j].mp_id;
            if (id < 0) continue;
            MapPoint* P = M->mp_by_id(id);
            if (!P) return fail("keypoint matched to unknown map point");
            K->mvpMapPoints[j] = P;
        }
    }
    return M;
}

size_t Map::snapshot_size() const {
    size_t n_kp = 0, n_cov = 0, n_obs = 0, n_gp = 0;
    for (const auto& K : mvKeyFrames) { n_kp += K->mvKeysUn.size(); n_cov += K->mvpOrderedConnectedKeyFrames.size(); }
    for (const auto& P : mvMapPoints) { n_obs += P->mObservations.size(); n_gp += P->mObservationsForGPBA.size(); }
    return pad8(sizeof(lbamap_header)) + pad8(sizeof(lbamap_cam) * nCamera) + pad8(sizeof(lbamap_kf) * mvKeyFrames.size()) +
           pad8(sizeof(lbamap_kp) * n_kp) + pad8(sizeof(int64_t) * n_cov) + pad8(sizeof(lbamap_mp) * mvMapPoints.size()) +
           pad8(sizeof(lbamap_mpobs) * n_obs) + pad8(sizeof(lbamap_gpobs) * n_gp);
}

int64_t Map::save(void* bytes, size_t cap) const {
    const size_t need = snapshot_size();
    if (cap < need) return -1;
    std::memset(bytes, 0, need);
    uint8_t* base = static_cast<uint8_t*>(bytes);
    size_t off = 0;
    auto put = [&](size_t sz) { uint8_t* p = base + off; off += pad8(sz); return p; };

    std::vector<lbamap_kp> kps;
    std::vector<int64_t> cov;
    std::vector<lbamap_kf> kfs(mvKeyFrames.size());
    for (size_t i = 0; i < mvKeyFrames.size(); ++i) {
        const MultiKeyFrame* K = mvKeyFrames[i].get();
        lbamap_kf& r = kfs[i];
        r.id = (int64_t)K->mnId;
        r.prev_id = K->mPrevKF ? (int64_t)K->mPrevKF->mnId : -1;
        r.next_id = K->mNextKF ? (int64_t)K->mNextKF->mnId : -1;
        r.time = K->mTimeStamp;
        for (int c = 0; c < nCamera; ++c) r.cam_time[c] = K->mvTimeStamps[c];
        const SE3f T = K->GetPose();
        std::memcpy(r.q, T.q, sizeof(r.q));
        std::memcpy(r.t, T.t, sizeof(r.t));
        std::memcpy(r.vel, K->GetVelocity(), sizeof(r.vel));
        r.bf = K->mbf;
        r.bad = K->mbBad;
        r.map_id = K->mMapId;
        r.kp_off = (int32_t)kps.size();
        r.n_kp = (int32_t)K->mvKeysUn.size();
        for (size_t j = 0; j < K->mvKeysUn.size(); ++j) {
            lbamap_kp kp{};
            kp.x = K->mvKeysUn[j].x; kp.y = K->mvKeysUn[j].y; kp.octave = K->mvKeysUn[j].octave;
            kp.cam = K->mmpKeyToCam[j]; kp.ur = K->mvuRight[j];
            kp.mp_id = K->mvpMapPoints[j] ? (int64_t)K->mvpMapPoints[j]->mnId : -1;
            kps.push_back(kp);
        }
        r.has_twc = 1;
        for (int c = 0; c < nCamera; ++c) {
            std::memcpy(r.twc_q[c], K->GetCameraPose(c).q, sizeof(r.twc_q[c]));
            std::memcpy(r.twc_t[c], K->GetCameraPose(c).t, sizeof(r.twc_t[c]));
        }
        r.covis_off = (int32_t)cov.size();
        r.n_covis = (int32_t)K->mvpOrderedConnectedKeyFrames.size();
        for (const MultiKeyFrame* C : K->mvpOrderedConnectedKeyFrames) cov.push_back((int64_t)C->mnId);
    }
    std::vector<lbamap_mp> mps(mvMapPoints.size());
    std::vector<lbamap_mpobs> mo;
    std::vector<lbamap_gpobs> go;
    for (size_t i = 0; i < mvMapPoints.size(); ++i) {
        const MapPoint* P = mvMapPoints[i].get();
        lbamap_mp& r = mps[i];
        r.id = (int64_t)P->mnId;
        r.pos[0] = P->mWorldPos.x; r.pos[1] = P->mWorldPos.y; r.pos[2] = P->mWorldPos.z;
        r.bad = P->mbBad;
        r.ref_kf = P->mpRefKF ? (int64_t)P->mpRefKF->mnId : -1;
        for (int c = 0; c < nCamera; ++c) r.track_depth[c] = P->mvTrackDepth[c];
        r.normal[0] = P->mNormalVector.x; r.normal[1] = P->mNormalVector.y; r.normal[2] = P->mNormalVector.z;
        r.min_dist = P->mfMinDistance;
        r.max_dist = P->mfMaxDistance;
        r.obs_off = (int32_t)mo.size();
        r.n_obs = (int32_t)P->mObservations.size();
        for (const auto& kv : P->mObservations) {
            lbamap_mpobs o{};
            o.kf_id = (int64_t)kv.first->mnId;
            for (int c = 0; c < LBAMAP_MAX_CAM; ++c) o.idx[c] = c < nCamera ? kv.second[c] : -1;
            mo.push_back(o);
        }
        r.gp_off = (int32_t)go.size();
        r.n_gp = (int32_t)P->mObservationsForGPBA.size();
        for (const auto& kv : P->mObservationsForGPBA) {
            lbamap_gpobs g{};
            g.kf_id = (int64_t)kv.first->mnId;
            g.time = kv.second.time; g.cam = kv.second.cam;
            g.x = kv.second.obs.x; g.y = kv.second.obs.y; g.octave = kv.second.obs.octave; g.ur = kv.second.ur;
            go.push_back(g);
        }
    }
    lbamap_header h{};
    std::memcpy(h.magic, "AMCSNAP", 8);
    h.version = LBAMAP_VERSION;
    h.n_cam = nCamera;
    h.n_kf = (int32_t)kfs.size();
    h.n_kp = (int32_t)kps.size();
    h.n_covis = (int32_t)cov.size();
    h.n_mp = (int32_t)mps.size();
    h.n_mpobs = (int32_t)mo.size();
    h.n_gpobs = (int32_t)go.size();
    h.n_levels = (int32_t)mvInvLevelSigma2.size();
    std::memcpy(h.qc, mQc, sizeof(h.qc));
    for (int l = 0; l < h.n_levels; ++l) { h.inv_level_sigma2[l] = mvInvLevelSigma2[l]; h.scale_factor[l] = mvScaleFactors[l]; }
    std::memcpy(put(sizeof(h)), &h, sizeof(h));
    std::vector<lbamap_cam> cams(nCamera);
    for (int c = 0; c < nCamera; ++c) {
        std::memcpy(cams[c].q, mCameras[c].Tbc.q, sizeof(cams[c].q));
        std::memcpy(cams[c].t, mCameras[c].Tbc.t, sizeof(cams[c].t));
        cams[c].fx = mCameras[c].fx; cams[c].fy = mCameras[c].fy; cams[c].cx = mCameras[c].cx; cams[c].cy = mCameras[c].cy;
        std::memcpy(cams[c].rbc_ini, mCameras[c].Rbc_ini, sizeof(cams[c].rbc_ini));
    }
    auto put_vec = [&](const void* src, size_t sz) { if (sz) std::memcpy(put(sz), src, sz); };
    put_vec(cams.data(), sizeof(lbamap_cam) * cams.size());
    put_vec(kfs.data(), sizeof(lbamap_kf) * kfs.size());
    put_vec(kps.data(), sizeof(lbamap_kp) * kps.size());
    put_vec(cov.data(), sizeof(int64_t) * cov.size());
    put_vec(mps.data(), sizeof(lbamap_mp) * mps.size());
    put_vec(mo.data(), sizeof(lbamap_mpobs) * mo.size());
    put_vec(go.data(), sizeof(lbamap_gpobs) * go.size());
    return (int64_t)off;
}

}  // namespace amc_slam
