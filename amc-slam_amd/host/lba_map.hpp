// lba_map.hpp — the slice of AMC-SLAM's map that Optimizer::LocalGPBA reads and writes.
//
// These classes keep the reference's names and semantics (include/KeyFrame.h:319-455,
// include/MapPoint.h:46-151, include/Map.h) for exactly the members LocalGPBA
// (src/Optimizer.cc:713-1432) touches, so the adapter in optimizer.cpp reads like the reference
// function.  They are host-side C++ (no Eigen / OpenCV / boost: those are absent here); the
// optimisation itself runs on the GPU through include/amc_lba.h.  Poses are float, as the
// reference stores them (Sophus::SE3f), and converted to double exactly where the reference does.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace amc_slam {

struct Vec3f {
    float x = 0, y = 0, z = 0;
};

// Sophus::SE3f: unit quaternion (x, y, z, w) + translation.
struct SE3f {
    float q[4] = {0, 0, 0, 1};
    float t[3] = {0, 0, 0};
    SE3f inverse() const;                       // Sophus se3.hpp:208-211 (float arithmetic)
    SE3f operator*(const SE3f& o) const;        // se3.hpp:304-308, so3.hpp:325-339 + renormalise
    Vec3f act(const Vec3f& p) const;            // so3.hpp:363-366 + translation
};

// SE3d with the same layout, the type the optimiser works in.
struct SE3d {
    double q[4] = {0, 0, 0, 1};
    double t[3] = {0, 0, 0};
    SE3d inverse() const;
    SE3f cast_float() const;                    // Sophus cast<float>(): per-coefficient cast + normalise
    static SE3d from_float(const SE3f& f);      // Sophus cast<double>()
};

struct KeyPoint {          // cv::KeyPoint fields LocalGPBA reads
    float x = 0, y = 0;
    int octave = 0;
};

class MultiKeyFrame;
class MapPoint;
class Map;

// GPObs (include/MapPoint.h:46-62): an observation from a non-keyframe frame between
// keyframe pKF and pKF->mNextKF, interpolated on the GP at `time`.
struct GPObs {
    double time = 0;
    int cam = 0;
    KeyPoint obs;
    float ur = -1;
    bool operator==(const GPObs& o) const {   // :58-61
        return time == o.time && cam == o.cam && obs.x == o.obs.x && obs.y == o.obs.y && ur == o.ur;
    }
};

struct CameraParams {      // Pinhole::mvParameters + MultiKeyFrame::mTbc[c]
    float fx = 0, fy = 0, cx = 0, cy = 0;
    SE3f Tbc;
    float Rbc_ini[4] = {0, 0, 0, 1};   // MultiFrame::mRbc_ini[c] (Sophus::SO3f, x y z w), src/Frame.cc:181
    float uncertainty2() const { return 1.0f; }   // Pinhole::uncertainty2 (src/CameraModels/Pinhole.cpp:56-59)
};

// std::map<MultiKeyFrame*, ...> ordered by keyframe id (see include/amc_lba_map.h "Ordering").
struct KFLess {
    bool operator()(const MultiKeyFrame* a, const MultiKeyFrame* b) const;
};

class MultiKeyFrame {
public:
    unsigned long mnId = 0;
    double mTimeStamp = 0;
    std::vector<double> mvTimeStamps;             // per camera
    int nCamera = 0;
    float mbf = 0;
    MultiKeyFrame* mPrevKF = nullptr;
    MultiKeyFrame* mNextKF = nullptr;
    unsigned long mnBALocalForKF = 0, mnBAFixedForKF = 0;
    unsigned long mnBAVertexStamp = 0;            // adapter: the window build that made this KF vertex mnBAVertex
    int mnBAVertex = -1;
    // global BA results held back while a loop is being corrected (include/KeyFrame.h:365-370)
    SE3f mTbwGBA;
    float mVwbGBA[6] = {0, 0, 0, 0, 0, 0};
    unsigned long mnBAGlobalForKF = 0;

    std::vector<KeyPoint> mvKeysUn;
    std::vector<int> mmpKeyToCam;
    std::vector<float> mvuRight;                  // indexed by keypoint (mmpGlobalToLocalID folded in)
    const std::vector<float>* mvInvLevelSigma2 = nullptr;
    const std::vector<float>* mvScaleFactors = nullptr;
    int mnScaleLevels = 0;
    const std::vector<CameraParams>* mvpCamera = nullptr;

    Map* GetMap() const { return mpMap; }
    bool isBad() const { return mbBad; }
    SE3f GetPose() const { return mTcw; }
    SE3f GetPoseInverse() const { return mTwc; }
    void SetPose(const SE3f& Tcw);                // KeyFrame::SetPose: caches the inverse and camera poses
    const float* GetVelocity() const { return mVel; }
    void SetVelocity(const float* v);
    Vec3f GetCameraCenter(int c) const;           // mTwc[c].translation() (src/KeyFrame.cc:203-207)
    const SE3f& GetCameraPose(int c) const { return mvTwc[c]; }
    void SetCachedPoses(const SE3f& Tbw, const std::vector<SE3f>& Twc);   // restore a snapshot's cache
    std::vector<MapPoint*> GetMapPointMatches() const { return mvpMapPoints; }
    std::vector<MultiKeyFrame*> GetVectorCovisibleKeyFrames() const { return mvpOrderedConnectedKeyFrames; }
    void EraseMapPointMatch(int idx);                          // src/KeyFrame.cc:364-368
    void EraseMapPointMatch(MapPoint* pMP, int cam);           // src/KeyFrame.cc:386-392

    // loader-side state
    Map* mpMap = nullptr;
    int mMapId = 0;
    bool mbBad = false;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<MultiKeyFrame*> mvpOrderedConnectedKeyFrames;

private:
    SE3f mTcw, mTwc;
    std::vector<SE3f> mvTwc;                      // per-camera Twc = Twb * Tbc
    float mVel[6] = {0, 0, 0, 0, 0, 0};
};

class MapPoint {
public:
    unsigned long mnId = 0;
    unsigned long mnBALocalForKF = 0;
    Vec3f mPosGBA;                      // global BA result held back during a loop correction
    unsigned long mnBAGlobalForKF = 0;  // (include/MapPoint.h)
    std::vector<float> mvTrackDepth;
    int nCamera = 0;

    bool isBad() const { return mbBad; }
    Vec3f GetWorldPos() const { return mWorldPos; }
    void SetWorldPos(const Vec3f& p) { mWorldPos = p; }
    std::map<MultiKeyFrame*, std::vector<int>, KFLess> GetObservations() const { return mObservations; }
    std::multimap<MultiKeyFrame*, GPObs, KFLess> GetGPObservations() const { return mObservationsForGPBA; }
    // the same containers by reference, for the window builds: the reference's accessors copy them under the
    // point's mutex (Tracking may add observations meanwhile); this map is read and changed only by the thread that
    // calls the adapter, so the builds read them in place (no map / multimap copy per point)
    const std::map<MultiKeyFrame*, std::vector<int>, KFLess>& ObservationsRef() const { return mObservations; }
    const std::multimap<MultiKeyFrame*, GPObs, KFLess>& GPObservationsRef() const { return mObservationsForGPBA; }
    std::vector<int> GetIndexInKeyFrame(MultiKeyFrame* pKF) const;
    void AddObservation(MultiKeyFrame* pKF, int idx);          // src/MapPoint.cc:196-229
    void EraseObservation(MultiKeyFrame* pKF, int c);           // src/MapPoint.cc:275-315
    void AddGPObservation(MultiKeyFrame* pKF, const GPObs& o);  // src/MapPoint.cc:317-321
    void EraseGPObservation(MultiKeyFrame* pKF, const GPObs& o); // src/MapPoint.cc:323-337
    void SetBadFlag();                                          // src/MapPoint.cc:356-386
    void UpdateNormalAndDepth();                                // src/MapPoint.cc:611-686
    int Observations() const { return nObs; }

    // loader-side state
    Map* mpMap = nullptr;
    bool mbBad = false;
    Vec3f mWorldPos;
    Vec3f mNormalVector;
    float mfMinDistance = 0, mfMaxDistance = 0;
    MultiKeyFrame* mpRefKF = nullptr;
    int nObs = 0;
    std::map<MultiKeyFrame*, std::vector<int>, KFLess> mObservations;
    std::multimap<MultiKeyFrame*, GPObs, KFLess> mObservationsForGPBA;
};

class Map {
public:
    // Map::KeyFramesInMap / GetMaxKFid / EraseMapPoint / IncreaseChangeIndex (src/Map.cc)
    long unsigned KeyFramesInMap() const;
    unsigned long GetMaxKFid() const { return mnMaxKFid; }
    // Map::GetAllKeyFrames / GetAllMapPoints (src/Map.cc): the map's sets, from which bad keyframes and
    // points have been erased (here they stay owned, flagged bad); keyframes of this map only, by id
    std::vector<MultiKeyFrame*> GetAllKeyFrames() const;
    std::vector<MapPoint*> GetAllMapPoints() const;
    // Map::GetInitKFid: the id of the keyframe the map was created with, i.e. its first (smallest) id
    // (the snapshot does not carry mnInitKFid; a map's ids grow from it)
    unsigned long GetInitKFid() const;
    void EraseMapPoint(MapPoint* pMP) { (void)pMP; }   // the point stays owned here, flagged bad
    void IncreaseChangeIndex() { ++mnBigChangeIdx; }
    std::mutex mMutexMapUpdate;

    MultiKeyFrame* kf_by_id(int64_t id) const;
    MapPoint* mp_by_id(int64_t id) const;

    // owned content
    int nCamera = 0;
    double mQc[36] = {};
    std::vector<CameraParams> mCameras;
    std::vector<float> mvInvLevelSigma2, mvScaleFactors;
    std::vector<std::unique_ptr<MultiKeyFrame>> mvKeyFrames;   // snapshot order
    std::vector<std::unique_ptr<MapPoint>> mvMapPoints;
    std::unordered_map<int64_t, MultiKeyFrame*> mKFById;
    std::unordered_map<int64_t, MapPoint*> mMPById;
    unsigned long mnMaxKFid = 0;
    int mnBigChangeIdx = 0;
    int mMapId = 0;

    // window snapshot I/O (include/amc_lba_map.h)
    static std::unique_ptr<Map> load(const void* bytes, size_t n, std::string* err);
    size_t snapshot_size() const;
    int64_t save(void* bytes, size_t cap) const;
};

}  // namespace amc_slam
