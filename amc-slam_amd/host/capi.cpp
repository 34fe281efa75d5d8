// capi.cpp — extern "C" entry points of include/amc_lba_map.h over the C++ adapter.
#include <cstring>
#include <exception>
#include <string>
#include <unordered_map>

#include "optimizer.hpp"

using amc_slam::Map;
using amc_slam::MultiKeyFrame;
using amc_slam::MapPoint;
using amc_slam::Optimizer;
using amc_slam::LocalGPBAWindow;

struct lbamap {
    std::unique_ptr<Map> map;
    lba_problem* problem = nullptr;
    int device = -1;
    std::string err;
};

extern "C" {

int lbamap_abi_version(void) { return LBAMAP_ABI_VERSION; }

int lbamap_load(lbamap** out, const void* bytes, size_t n_bytes) {
    if (!out || !bytes) return LBA_E_ARG;
    *out = nullptr;
    auto* m = new lbamap();
    m->map = Map::load(bytes, n_bytes, &m->err);
    if (!m->map) {
        delete m;
        return LBA_E_ARG;
    }
    *out = m;
    return LBA_OK;
}

void lbamap_free(lbamap* m) {
    if (!m) return;
    if (m->problem) lba_destroy(m->problem);
    delete m;
}

const char* lbamap_last_error(const lbamap* m) { return m ? m->err.c_str() : "null map"; }

size_t lbamap_snapshot_size(const lbamap* m) { return m ? m->map->snapshot_size() : 0; }

int64_t lbamap_save(const lbamap* m, void* bytes, size_t cap) {
    if (!m || !bytes) return LBA_E_ARG;
    const int64_t n = m->map->save(bytes, cap);
    return n < 0 ? LBA_E_ARG : n;
}

int lbamap_local_gpba(lbamap* m, int64_t kf_id, volatile const int32_t* stop_flag, const lbamap_options* opt,
                      lbamap_result* out) {
    (void)stop_flag;   // handed to g2o only after optimize() in the reference (Optimizer.cc:1254-1255)
    if (!m || !opt) return LBA_E_ARG;
    MultiKeyFrame* K = m->map->kf_by_id(kf_id);
    if (!K) {
        m->err = "unknown keyframe id";
        return LBA_E_ARG;
    }
    try {
        if (m->problem && m->device != opt->device) {
            lba_destroy(m->problem);
            m->problem = nullptr;
        }
        if (!m->problem) {
            lba_config cfg{};
            cfg.device = opt->device;
            const int rc = lba_create(&m->problem, &cfg);
            if (rc != LBA_OK) {
                m->problem = nullptr;
                m->err = "lba_create failed";
                return rc;
            }
            m->device = opt->device;
        }
        const int rc = Optimizer::LocalGPBA(K, m->map.get(), *opt, m->problem, out);
        if (rc < 0 && rc != LBA_E_DIVERGED) m->err = lba_last_error(m->problem);
        return rc;
    } catch (const std::exception& e) {
        m->err = e.what();
        return LBA_E_ARG;
    }
}

static int ensure_problem(lbamap* m, int device) {
    if (m->problem && m->device != device) {
        lba_destroy(m->problem);
        m->problem = nullptr;
    }
    if (!m->problem) {
        lba_config cfg{};
        cfg.device = device;
        const int rc = lba_create(&m->problem, &cfg);
        if (rc != LBA_OK) {
            m->problem = nullptr;
            m->err = "lba_create failed";
            return rc;
        }
        m->device = device;
    }
    return LBA_OK;
}

int lbamap_global_ba(lbamap* m, int32_t n_iterations, volatile const int32_t* stop_flag, uint64_t loop_kf,
                     const lbamap_options* opt, lbamap_ba_result* out) {
    if (!m || !opt || n_iterations < 0) return LBA_E_ARG;
    try {
        int rc = ensure_problem(m, opt->device);
        if (rc != LBA_OK) return rc;
        const std::vector<MultiKeyFrame*> vpKFs = m->map->GetAllKeyFrames();   // (src/Optimizer.cc:55-57)
        const std::vector<MapPoint*> vpMP = m->map->GetAllMapPoints();
        if (vpKFs.empty()) {
            m->err = "the map has no keyframes";
            return LBA_E_ARG;
        }
        rc = Optimizer::BundleAdjustment(vpKFs, vpMP, n_iterations, stop_flag, (unsigned long)loop_kf, *opt, m->problem,
                                         out);
        if (rc < 0) m->err = lba_last_error(m->problem);
        return rc;
    } catch (const std::exception& e) {
        m->err = e.what();
        return LBA_E_ARG;
    }
}

int lbamap_global_ba_thread(lbamap* m, int32_t n_iterations, bool* stop, uint64_t loop_kf) {
    if (!m || n_iterations < 0) return LBA_E_ARG;
    try {
        Optimizer::GlobalBundleAdjustemnt(m->map.get(), n_iterations, stop, (unsigned long)loop_kf, true);
        return LBA_OK;
    } catch (const std::exception& e) {
        m->err = e.what();
        return LBA_E_ARG;
    }
}

int lbamap_kf_gba(const lbamap* m, int64_t kf_id, float q[4], float t[3], float vel[6], uint64_t* loop_kf) {
    if (!m) return LBA_E_ARG;
    const MultiKeyFrame* K = m->map->kf_by_id(kf_id);
    if (!K) return LBA_E_ARG;
    if (q) std::memcpy(q, K->mTbwGBA.q, 4 * sizeof(float));
    if (t) std::memcpy(t, K->mTbwGBA.t, 3 * sizeof(float));
    if (vel) std::memcpy(vel, K->mVwbGBA, 6 * sizeof(float));
    if (loop_kf) *loop_kf = K->mnBAGlobalForKF;
    return LBA_OK;
}

int lbamap_mp_gba(const lbamap* m, int64_t mp_id, float pos[3], uint64_t* loop_kf) {
    if (!m) return LBA_E_ARG;
    const MapPoint* P = m->map->mp_by_id(mp_id);
    if (!P) return LBA_E_ARG;
    if (pos) { pos[0] = P->mPosGBA.x; pos[1] = P->mPosGBA.y; pos[2] = P->mPosGBA.z; }
    if (loop_kf) *loop_kf = P->mnBAGlobalForKF;
    return LBA_OK;
}

int lbamap_build_ba_window(lbamap* m, int32_t counts[6], lba_kf* kfs, double* lm_xyz, lba_obs* obs, lba_prior* priors,
                           int32_t* vel_kfs, lba_cam* cams, int64_t* kf_ids, int64_t* mp_ids, int32_t* obs_tag,
                           lba_config* cfg) {
    if (!m || !counts) return LBA_E_ARG;
    amc_slam::BundleAdjustmentWindow W;
    Optimizer::BuildBundleAdjustmentWindow(m->map->GetAllKeyFrames(), m->map->GetAllMapPoints(), &W);
    counts[0] = (int32_t)W.kfs.size();
    counts[1] = (int32_t)W.mp_ids.size();
    counts[2] = (int32_t)W.obs.size();
    counts[3] = (int32_t)W.priors.size();
    counts[4] = (int32_t)W.vel_kfs.size();
    counts[5] = (int32_t)W.cams.size();
    auto cp = [](void* dst, const void* src, size_t n) { if (dst && n) std::memcpy(dst, src, n); };
    cp(kfs, W.kfs.data(), sizeof(lba_kf) * W.kfs.size());
    cp(lm_xyz, W.lm.data(), sizeof(double) * W.lm.size());
    cp(obs, W.obs.data(), sizeof(lba_obs) * W.obs.size());
    cp(priors, W.priors.data(), sizeof(lba_prior) * W.priors.size());
    cp(vel_kfs, W.vel_kfs.data(), sizeof(int32_t) * W.vel_kfs.size());
    cp(cams, W.cams.data(), sizeof(lba_cam) * W.cams.size());
    cp(kf_ids, W.kf_ids.data(), sizeof(int64_t) * W.kf_ids.size());
    cp(mp_ids, W.mp_ids.data(), sizeof(int64_t) * W.mp_ids.size());
    cp(obs_tag, W.obs_tag.data(), sizeof(int32_t) * W.obs_tag.size());
    if (cfg) *cfg = W.cfg;
    return LBA_OK;
}

int lbamap_build_window(lbamap* m, int64_t kf_id, const lbamap_options* opt, int32_t counts[6], lba_kf* kfs,
                        double* lm_xyz, lba_obs* obs, lba_prior* priors, int32_t* vel_kfs, lba_cam* cams,
                        int64_t* kf_ids, int64_t* mp_ids, int32_t* obs_tag, lba_config* cfg) {
    if (!m || !opt || !counts) return LBA_E_ARG;
    MultiKeyFrame* K = m->map->kf_by_id(kf_id);
    if (!K) {
        m->err = "unknown keyframe id";
        return LBA_E_ARG;
    }
    // dry run: remember the BA flags and restore them afterwards
    std::vector<std::pair<unsigned long, unsigned long>> kf_flags;
    std::vector<unsigned long> mp_flags;
    for (const auto& k : m->map->mvKeyFrames) kf_flags.push_back({k->mnBALocalForKF, k->mnBAFixedForKF});
    for (const auto& p : m->map->mvMapPoints) mp_flags.push_back(p->mnBALocalForKF);
    LocalGPBAWindow W;
    Optimizer::BuildLocalGPBAWindow(K, opt->large != 0, &W);
    for (size_t i = 0; i < kf_flags.size(); ++i) {
        m->map->mvKeyFrames[i]->mnBALocalForKF = kf_flags[i].first;
        m->map->mvKeyFrames[i]->mnBAFixedForKF = kf_flags[i].second;
    }
    for (size_t i = 0; i < mp_flags.size(); ++i) m->map->mvMapPoints[i]->mnBALocalForKF = mp_flags[i];

    counts[0] = (int32_t)W.kfs.size();
    counts[1] = (int32_t)W.mp_ids.size();
    counts[2] = (int32_t)W.obs.size();
    counts[3] = (int32_t)W.priors.size();
    counts[4] = (int32_t)W.vel_kfs.size();
    counts[5] = (int32_t)W.cams.size();
    auto cp = [](void* dst, const void* src, size_t n) { if (dst && n) std::memcpy(dst, src, n); };
    cp(kfs, W.kfs.data(), sizeof(lba_kf) * W.kfs.size());
    cp(lm_xyz, W.lm.data(), sizeof(double) * W.lm.size());
    cp(obs, W.obs.data(), sizeof(lba_obs) * W.obs.size());
    cp(priors, W.priors.data(), sizeof(lba_prior) * W.priors.size());
    cp(vel_kfs, W.vel_kfs.data(), sizeof(int32_t) * W.vel_kfs.size());
    cp(cams, W.cams.data(), sizeof(lba_cam) * W.cams.size());
    cp(kf_ids, W.kf_ids.data(), sizeof(int64_t) * W.kf_ids.size());
    cp(mp_ids, W.mp_ids.data(), sizeof(int64_t) * W.mp_ids.size());
    cp(obs_tag, W.obs_tag.data(), sizeof(int32_t) * W.obs_tag.size());
    if (cfg) *cfg = W.cfg;
    return LBA_OK;
}

}  // extern "C"
