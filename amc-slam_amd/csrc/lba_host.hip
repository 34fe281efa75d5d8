// lba_host.hip — host side of the MI355X local BA: window preprocessing into the HBM layout of
// lba_device.hpp, the Levenberg-Marquardt driver (g2o OptimizationAlgorithmLevenberg semantics,
// Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-194) and the C ABI of
// include/amc_lba.h.
//
// State stays resident on the device between LM trials: the current and trial estimates are two
// buffers, so g2o's push/pop/discardTop (sparse_optimizer.cpp:589-613) become a buffer swap.
// The host reads back four doubles per trial (chi2 before, chi2 after, computeScale, factor status).
#include <rccl/rccl.h>

#include <algorithm>
#include <sched.h>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <queue>
#include <limits>
#include <map>
#include <string>
#include <exception>
#include <functional>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/amc_lba.h"
#include "lba_device.hpp"
#include "lba_plan.hpp"
#include "lba_math.hpp"

using namespace lba;

// the last panel pattern an engine planned (plan_panels_cached)
struct PlanCache {
    int NP = -1, NPk = -1;
    std::string env;   // (the diagnostics' LBA_ND_* settings it was made under)
    std::vector<std::vector<int>> lower;
    lba_plan::Plan plan;
};

struct lba_problem {
    lba_config cfg{};
    std::string err;
    hipStream_t stream = nullptr;
    hipEvent_t ev[10] = {};
    bool has_problem = false;
    bool linearized = false;
    int n_kf = 0, n_lm = 0, n_obs = 0, n_cam = 0;
    std::vector<int> kf_hidx;     // per KF: pose block or -1
    std::vector<int> lm_dev;      // original landmark -> device index (-1 inactive)
    std::vector<int> lm_orig;     // device index -> original landmark
    std::vector<int> obs_dev;     // original observation -> device index
    std::vector<double> lm_host;  // original landmark positions (inactive ones are returned as is)
    std::vector<int> kf_fixed;
    int n_lm_dev = 0, n_pb = 0, np = 0;
    // free extrinsics: KF slots n_kf .. n_kf + n_ext - 1, pose blocks after the KFs' (12 wide, the second
    // half inert); the caller's pose system has them 6 wide: pose_ext[i] = caller index of internal pose
    // index i (-1: inert), np_ext = its dimension
    int n_ext = 0, np_ext = 0;
    std::vector<int> pose_ext;
    std::vector<lba_cam> cams;
    std::vector<int> ext_cams;
    DevProblem D{};
    double* kst[2] = {nullptr, nullptr};
    double* lst[2] = {nullptr, nullptr};
    int cur = 0;
    int nd_tail = 0;              // panels of the dissection's tail separator (rows reaching back: loops)
    int chain = 0;                // panels on the factorisation's dependent chain
    int nd_levels = 0;            // depth of the nested dissection
    int s_tiles = 0;              // tiles of the lower triangle of S (the pattern before fill-in)
    double flops_factor = 0.0;    // algorithmic FLOPs of the tile factorisation (symbolic structure of L)
    bool host_only = false;       // lba_setup_host_profile: stop set_problem after the host preprocessing
    uint32_t setup_hash = 0;      // (host_only) fingerprint of the tiling / slab layout
    int setup_tiles = 0;
    std::vector<double> setup_ms; // wall time of the set-up phases (order/pairs, tiles, slots/state, ...)
    PlanCache plan_cache;
    // device buffers of the window, in set_problem's allocation order; the next set_problem reuses
    // them in the same order where they are large enough (LocalGPBA windows are alike call to call),
    // so a call pays no hipMalloc / hipFree
    struct Alloc { void* ptr; size_t bytes; };
    std::vector<Alloc> allocs;
    size_t alloc_cursor = 0;
    // pinned staging of the uploads (persistent chunks, bump-allocated per set_problem): dupload copies
    // a host array into it and queues the host->device copy on the stream, so the DMA overlaps the rest
    // of the preprocessing; the next set_problem reuses it after its stream synchronisation
    std::vector<Alloc> pin_chunks;
    size_t pin_chunk = 0, pin_off = 0;
    // the window's read-only arrays (dupload): bump-allocated in persistent device chunks, each with a pinned mirror;
    // an array is copied into the mirror at its offset and the staged range since the last flush goes out as ONE
    // host->device copy per chunk at every phase boundary (flush_uploads), instead of one copy per array (~65 per
    // set-up, each a runtime call)
    std::vector<Alloc> up_dev, up_pin;
    std::vector<size_t> up_end;             // bytes staged in each chunk this set-up (the current one: up_off)
    size_t up_chunk = 0, up_off = 0;        // allocation position
    size_t up_fchunk = 0, up_foff = 0;      // flushed up to here
    // observation-sized host scratch arrays of set_problem, kept between calls: resizing to the same
    // length touches nothing (no allocation, page faults or zeroing per window; every element is written)
    std::vector<int> scr_i[16];
    std::vector<double> scr_d[2];
    // device ranges set_problem zeroes: collected, then cleared by ONE kernel launch at its end (k_zero_ranges)
    // instead of one hipMemsetAsync each (~17 runtime calls and ~28 fill kernels per set-up)
    std::vector<unsigned long long> zero_list;   // pairs: device address, 4-byte words
    double* h_fin = nullptr;      // host-mapped coherent [HFIN_DOUBLES]: trial summary [4], sequence
                                  // number [4], LMCtl mirror [8..] (queued optimisation)
    double* d_hfin = nullptr;     // its device address
    int* h_log = nullptr;         // host-mapped [HLOG_CAP]: per queued trial, 1 if it relinearised
    int* d_hlog = nullptr;
    std::vector<hipEvent_t> qev;  // queued optimisation, LBA_FLAG_TIME_SWEEP: 2 events per trial
    size_t s_bytes = 0;           // device bytes of S + L (packed envelopes)
    unsigned long long fin_seq = 0;
    unsigned cf_epoch = 0;        // launches of the dataflow factorisation (its flags hold the epoch)
    unsigned upd_epoch = 0;       // launches of k_update (the fused evaluation's producer flags hold the epoch)
    unsigned asm_epoch = 0;       // launches of k_exp_asm (its expansions' flags hold the epoch)
    bool gps_fresh[2] = {false, false};   // state buffer s has its pose samples with Jacobian factors
    double lambda = -1.0, ni = 2.0;
    int nBad = 0;
    // partitioned global BA (lba_set_partition): the caller's sum all-reduce across ranks
    int part_rank = 0, part_n = 0;
    std::vector<int> split_own;       // distributed factorisation: owner rank of each factorisation panel, -1 top
    std::vector<int> ppos_h;          // natural panel -> factorisation position
    int split_tasks[2] = {0, 0};      // tasks of its two launches on this rank
    int split_panels[2] = {0, 0};     // panels of this rank's subtree / of the top
    double flops_factor_rank = 0.0;   // factorisation FLOPs of this rank (its subtree + the top; all when replicated)
    lba_allreduce_fn red_fn = nullptr;
    void* red_user = nullptr;
    ncclComm_t comm = nullptr;        // owned when set by lba_set_partition_rccl
    double* d_status = nullptr;       // set-up status word of the partition (part_status)
    bool status_entered = false;      // this set_problem has reached the status all-reduce
    void* group_slot = nullptr;       // owned (rank, group) record of lba_set_partition_group
    // window farm (lba_set_farm*, lba_farm_plan, lba_farm_exchange): the collective and the exchange plan
    int farm_rank = 0, farm_n = 0;
    lba_allreduce_fn farm_fn = nullptr;   // sum all-reduce (the all-gather over zero-padded slots)
    void* farm_user = nullptr;
    ncclComm_t farm_comm = nullptr;       // owned, lba_set_farm_rccl: native in-place all-gather
    void* farm_slot = nullptr;            // owned GroupSlot of lba_set_farm_group
    bool farm_planned = false;
    int f_stride = 0, f_kcap = 0, f_npk = 0, f_npl = 0, f_nrk = 0, f_nrl = 0;
    double* f_buf = nullptr;              // [farm_n][f_stride]: published keyframes (kcap x FARM_KF), landmarks
    size_t f_buf_bytes = 0;
    int* f_idx = nullptr;                 // published KFs | published landmarks | (dst, src) KFs | (dst, src) lms
    size_t f_idx_bytes = 0;
};

namespace {

constexpr int HFIN_DOUBLES = 8 + LMCTL_DOUBLES;

struct HipError {
    hipError_t e;
    const char* what;
};

#define HIPCHK(x)                                   \
    do {                                            \
        hipError_t _e = (x);                        \
        if (_e != hipSuccess) throw HipError{_e, #x}; \
    } while (0)

struct ApiError {
    int code;
    std::string msg;
};

// the caller's all-reduce (sum, in place, enqueued on the problem's stream)
void preduce(lba_problem* p, double* buf, int64_t n) {
    if (p->red_fn(buf, n, (void*)p->stream, p->red_user) != 0)
        throw ApiError{LBA_E_HIP, "partition all-reduce failed"};
}

// The factorisation plan of a panel pattern (lba_set_problem and lba_partition_assign must agree on it).
// (diagnostics: LBA_ND_LEVELS=<n> caps the dissection depth, 0 = natural order; LBA_ND_NO_TAIL; LBA_ND_METHOD=1
// the interval dissection only, 2 the graph dissection only)
lba_plan::Plan plan_panels(int NP, int NPk, const std::vector<std::vector<int>>& lower) {
    const char* lv = std::getenv("LBA_ND_LEVELS");
    const char* nm = std::getenv("LBA_ND_METHOD");
    return lba_plan::make_plan(NP, NPk, lower, lv ? std::atoi(lv) : 64, std::getenv("LBA_ND_NO_TAIL") == nullptr, 16,
                               nm ? std::atoi(nm) : 0);
}
// The same, remembering the last pattern planned on this engine: consecutive windows of a LocalGPBA sequence
// usually couple their keyframes in the same band pattern, and the plan is a function of (NP, NPk, pattern) and the
// diagnostics' environment alone (so a hit returns exactly what make_plan would)
const lba_plan::Plan& plan_panels_cached(PlanCache& c, int NP, int NPk, const std::vector<std::vector<int>>& lower) {
    std::string env;
    for (const char* k : {"LBA_ND_LEVELS", "LBA_ND_METHOD", "LBA_ND_NO_TAIL"}) {
        const char* v = std::getenv(k);
        env += v ? std::string(v) + ";" : std::string("-;");
    }
    if (c.NP == NP && c.NPk == NPk && c.env == env && c.lower == lower) return c.plan;
    c.plan = plan_panels(NP, NPk, lower);
    c.NP = NP;
    c.NPk = NPk;
    c.env = env;
    c.lower = lower;
    return c.plan;
}

// Partitioned set-up: every rank reports the outcome of its host preprocessing in one all-reduce at a
// fixed point ahead of the first collective, so a rank that failed (argument check, tile limits ...)
// releases its peers instead of leaving them in a collective it never reaches: every rank then fails.
void part_status(lba_problem* p, int failed) {
    p->status_entered = true;
    const double v = failed ? 1.0 : 0.0;
    HIPCHK(hipMemcpy(p->d_status, &v, sizeof(double), hipMemcpyHostToDevice));
    preduce(p, p->d_status, 1);
    HIPCHK(hipStreamSynchronize(p->stream));
    double sum = 0.0;
    HIPCHK(hipMemcpy(&sum, p->d_status, sizeof(double), hipMemcpyDeviceToHost));
    if (sum != 0.0 && !failed) throw ApiError{LBA_E_ARG, "another rank of the partition failed its set-up"};
}
// a failing set-up that has not reached the status point yet reports its failure there
void release_peers(lba_problem* p) {
    if (p->part_n <= 0 || p->status_entered || !p->d_status) return;
    try {
        part_status(p, 1);
    } catch (...) {
    }
}

// LBA_PHASE_TIMING=<file>: dump the per-workgroup phase stamps of the last k_linearize / k_schur
// launch and the tile shapes (diagnostics; scripts/phase_times.py reads it)
void dump_phase_times(lba_problem* p) {
    const DevProblem& D = p->D;
    const char* path = std::getenv("LBA_PHASE_TIMING");
    if (!path || !D.tdbg_lin || D.n_tiles <= 0) return;
    const size_t n = (size_t)D.n_tiles * 16;
    std::vector<unsigned long long> lin(n), sch(n);
    const int* cols[6] = {D.tile_nobs, D.tile_nsmp, D.tile_npair, D.tile_nlm, D.tile_nsent, D.tile_nkf};
    std::vector<int> shape(6 * (size_t)D.n_tiles);
    if (hipDeviceSynchronize() != hipSuccess) return;
    (void)hipMemcpy(lin.data(), D.tdbg_lin, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(sch.data(), D.tdbg_schur, n * 8, hipMemcpyDeviceToHost);
    for (int c = 0; c < 6; ++c)
        (void)hipMemcpy(shape.data() + (size_t)c * D.n_tiles, cols[c], 4 * (size_t)D.n_tiles, hipMemcpyDeviceToHost);
    const int nblk = D.npad / CHOL_NB + 1;
    std::vector<unsigned long long> ch((size_t)nblk * 16), bs((size_t)nblk * 16);
    (void)hipMemcpy(ch.data(), D.tdbg_chol, ch.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(bs.data(), D.tdbg_bs, bs.size() * 8, hipMemcpyDeviceToHost);
    std::vector<unsigned long long> cft((size_t)4096 * CF_TDBG_STRIDE);
    (void)hipMemcpy(cft.data(), D.tdbg_cf, cft.size() * 8, hipMemcpyDeviceToHost);
    if (FILE* f = std::fopen(path, "wb")) {
        const int nt = D.n_tiles;
        std::fwrite(&nt, 4, 1, f);
        std::fwrite(lin.data(), 8, n, f);
        std::fwrite(sch.data(), 8, n, f);
        std::fwrite(shape.data(), 4, shape.size(), f);
        std::fwrite(&nblk, 4, 1, f);
        std::fwrite(ch.data(), 8, ch.size(), f);
        std::fwrite(bs.data(), 8, bs.size(), f);
        std::fwrite(cft.data(), 8, cft.size(), f);
        std::fclose(f);
    }
}

void release_all(lba_problem* p) {   // (lba_destroy)
    for (auto& a : p->allocs) (void)hipFree(a.ptr);
    p->allocs.clear();
    p->alloc_cursor = 0;
    for (auto& a : p->up_dev) (void)hipFree(a.ptr);
    for (auto& a : p->up_pin) (void)hipHostFree(a.ptr);
    p->up_dev.clear();
    p->up_pin.clear();
    p->up_end.clear();
    p->up_chunk = p->up_off = p->up_fchunk = p->up_foff = 0;
}

void free_all(lba_problem* p) {   // the buffers stay allocated for the next window's dalloc calls
    dump_phase_times(p);
    p->alloc_cursor = 0;
    p->pin_chunk = 0;
    p->pin_off = 0;
    p->up_chunk = p->up_off = p->up_fchunk = p->up_foff = 0;
    p->kst[0] = p->kst[1] = p->lst[0] = p->lst[1] = nullptr;
    p->D = DevProblem{};
    p->has_problem = false;
    p->linearized = false;
}

template <typename T>
T* dalloc(lba_problem* p, size_t n) {
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    if (p->alloc_cursor < p->allocs.size()) {
        auto& a = p->allocs[p->alloc_cursor];
        if (a.bytes < bytes) {
            (void)hipFree(a.ptr);
            a.ptr = nullptr;
            a.bytes = 0;
            HIPCHK(hipMalloc(&a.ptr, bytes));
            a.bytes = bytes;
        }
        ++p->alloc_cursor;
        return static_cast<T*>(a.ptr);
    }
    void* d = nullptr;
    HIPCHK(hipMalloc(&d, bytes));
    p->allocs.push_back({d, bytes});
    p->alloc_cursor = p->allocs.size();
    return static_cast<T*>(d);
}
// bytes of pinned staging (16-byte aligned) from the persistent chunks
void* pin_stage(lba_problem* p, size_t bytes) {
    bytes = (bytes + 15) & ~(size_t)15;
    while (true) {
        if (p->pin_chunk == p->pin_chunks.size()) {
            lba_problem::Alloc a{nullptr, std::max<size_t>(bytes, (size_t)16 << 20)};
            HIPCHK(hipHostMalloc(&a.ptr, a.bytes, hipHostMallocDefault));
            p->pin_chunks.push_back(a);
        }
        lba_problem::Alloc& a = p->pin_chunks[p->pin_chunk];
        if (p->pin_off + bytes <= a.bytes) {
            void* r = static_cast<char*>(a.ptr) + p->pin_off;
            p->pin_off += bytes;
            return r;
        }
        ++p->pin_chunk;
        p->pin_off = 0;
    }
}
// v into the device buffer d (at least v.size() elements), through the pinned staging chunks, asynchronously on the
// problem's stream
template <typename T>
void upload_into(lba_problem* p, T* d, const std::vector<T>& v) {
    if (!v.empty()) {
        const size_t bytes = v.size() * sizeof(T);
        void* st = pin_stage(p, bytes);
        if (bytes >= ((size_t)1 << 19)) {   // large arrays: the copy into pinned memory in 8 pieces
            par_for(8, [&](int piece) {
                const size_t b0 = bytes * piece / 8, b1 = bytes * (piece + 1) / 8;
                std::memcpy(static_cast<char*>(st) + b0, reinterpret_cast<const char*>(v.data()) + b0, b1 - b0);
            });
        } else {
            std::memcpy(st, v.data(), bytes);
        }
        HIPCHK(hipMemcpyAsync(d, st, bytes, hipMemcpyHostToDevice, p->stream));
    }
}
// the staged part of the upload chunks since the last flush, one host->device copy per chunk
void flush_uploads(lba_problem* p) {
    while (p->up_fchunk < p->up_pin.size() && (p->up_fchunk < p->up_chunk || p->up_foff < p->up_off)) {
        const size_t end = p->up_fchunk < p->up_chunk ? p->up_end[p->up_fchunk] : p->up_off;
        if (end > p->up_foff)
            HIPCHK(hipMemcpyAsync(static_cast<char*>(p->up_dev[p->up_fchunk].ptr) + p->up_foff,
                                  static_cast<char*>(p->up_pin[p->up_fchunk].ptr) + p->up_foff, end - p->up_foff,
                                  hipMemcpyHostToDevice, p->stream));
        if (p->up_fchunk < p->up_chunk) {
            ++p->up_fchunk;
            p->up_foff = 0;
        } else {
            p->up_foff = end;
        }
    }
}
template <typename T>
T* dupload(lba_problem* p, const std::vector<T>& v) {
    const size_t bytes = ((std::max<size_t>(v.size(), 1) * sizeof(T)) + 255) & ~(size_t)255;
    while (true) {
        if (p->up_chunk == p->up_dev.size()) {
            lba_problem::Alloc dv{nullptr, std::max<size_t>(bytes, (size_t)32 << 20)}, pn{nullptr, dv.bytes};
            HIPCHK(hipMalloc(&dv.ptr, dv.bytes));
            HIPCHK(hipHostMalloc(&pn.ptr, pn.bytes, hipHostMallocDefault));
            p->up_dev.push_back(dv);
            p->up_pin.push_back(pn);
            p->up_end.push_back(0);
        }
        if (p->up_off + bytes <= p->up_dev[p->up_chunk].bytes) break;
        p->up_end[p->up_chunk] = p->up_off;   // (the rest of this chunk stays unused)
        ++p->up_chunk;
        p->up_off = 0;
    }
    char* st = static_cast<char*>(p->up_pin[p->up_chunk].ptr) + p->up_off;
    T* d = reinterpret_cast<T*>(static_cast<char*>(p->up_dev[p->up_chunk].ptr) + p->up_off);
    p->up_off += bytes;
    const size_t nb = v.size() * sizeof(T);
    if (nb >= ((size_t)1 << 19)) {   // large arrays: the copy into pinned memory in 8 pieces
        par_for(8, [&](int piece) {
            const size_t b0 = nb * piece / 8, b1 = nb * (piece + 1) / 8;
            std::memcpy(st + b0, reinterpret_cast<const char*>(v.data()) + b0, b1 - b0);
        });
    } else if (nb) {
        std::memcpy(st, v.data(), nb);
    }
    return d;
}

// f(i) for i in [0, n) on up to SETUP_THREADS_MAX (16) host threads, at most the CPUs this process may run on
// (LBA_SETUP_THREADS overrides; 1: serial).  Round 3 measured 16 threads no faster than 8
// (profiles/r3ai_setup_threads.txt); round 4's parallel tile-list concatenation and device-order records made
// the 16-piece passes scale, and 16 is the default since (profiles/r4z_setup_phases.txt).  Callers split work into a fixed number of pieces, so the
// results never depend on the thread count.  The workers persist (a set-up makes a dozen parallel passes;
// spawning threads per pass cost ~0.1 ms each) and, after a pass, poll for the next one for a while before
// they sleep: a set-up's passes follow each other within a millisecond, and an OS wake-up of the workers per
// pass cost more than many of the passes themselves.  Pieces are claimed from one counter that packs
// (pass, piece), so a worker that arrives late takes no piece of a later pass for an earlier one; the caller
// waits for the pieces to be finished, not for every worker to have looked in.  A pass that finds the pool
// busy (another problem setting up on another thread) runs on its caller's thread alone.
constexpr int SETUP_THREADS_MAX = 16;
// the fixed number of pieces every parallel pass of the set-up splits its work into (the results do not depend on
// the thread count; tiles never straddle a piece boundary)
constexpr int SETUP_PIECES = 16;
class SetupPool {
  public:
    static SetupPool& get() {
        static SetupPool pool;
        return pool;
    }
    int size() const { return (int)workers_.size() + 1; }
    // false: the pool is in use (the caller runs the pass itself)
    template <class F>
    bool run(int n, F& f) {
        std::unique_lock<std::mutex> busy(busy_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        std::function<void(int)> job = [&](int i) { f(i); };
        job_ = &job;
        n_.store(n, std::memory_order_relaxed);
        done_.store(0, std::memory_order_relaxed);
        err_ = nullptr;
        const unsigned long long g = ++pass_;
        {
            std::lock_guard<std::mutex> lk(m_);
            claim_.store(g << 32, std::memory_order_release);   // publishes job_ / n_ with the pass number
        }
        cv_.notify_all();
        work(g);   // the caller takes pieces too
        for (int spins = 0; done_.load(std::memory_order_acquire) < n; ++spins)
            if (spins > 4096) std::this_thread::yield();
        // close the pass before any field of the next one is written: a worker that loaded this pass's
        // last claim word (every piece taken) and was preempted before its bound check would otherwise
        // pass that check against the next pass's larger n_ and win its CAS against the unchanged word,
        // running a piece of the next job ahead of its publication
        claim_.store((g << 32) | CLOSED, std::memory_order_release);
        job_ = nullptr;
        if (err_) std::rethrow_exception(err_);
        return true;
    }

  private:
    static constexpr int POLL_US = 3000;   // how long an idle worker polls for the next pass before it sleeps
    static constexpr unsigned long long CLOSED = 0x7fffffffull;   // piece word of a finished pass (>= any n)
    SetupPool() {
        const char* e = std::getenv("LBA_SETUP_THREADS");
        const int v = e ? std::atoi(e) : 0;
        int avail = (int)std::thread::hardware_concurrency();
        cpu_set_t cs;
        if (sched_getaffinity(0, sizeof(cs), &cs) == 0) avail = std::min(avail > 0 ? avail : CPU_COUNT(&cs), CPU_COUNT(&cs));
        const int nt = v > 0 ? v : std::max(1, std::min(SETUP_THREADS_MAX, avail));
        for (int t = 1; t < nt; ++t)
            workers_.emplace_back([this] {
                unsigned long long seen = 0;
                while (true) {
                    auto fresh = [&] { return stop_.load(std::memory_order_acquire) ||
                                              (claim_.load(std::memory_order_acquire) >> 32) != seen; };
                    const auto t0 = std::chrono::steady_clock::now();
                    while (!fresh()) {
                        for (int k = 0; k < 64 && !fresh(); ++k) __builtin_ia32_pause();
                        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(POLL_US)) {
                            std::unique_lock<std::mutex> lk(m_);
                            cv_.wait(lk, fresh);
                        }
                    }
                    if (stop_.load(std::memory_order_acquire)) return;
                    seen = claim_.load(std::memory_order_acquire) >> 32;
                    work(seen);
                }
            });
    }
    ~SetupPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_.store(true, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }
    // claim pieces of pass g until none is left (or the pass is over); every piece claimed is counted done
    void work(unsigned long long g) {
        for (;;) {
            unsigned long long c = claim_.load(std::memory_order_acquire);
            int i;
            do {
                if ((c >> 32) != g || (int)(c & 0xffffffffu) >= n_.load(std::memory_order_relaxed)) return;
                i = (int)(c & 0xffffffffu);
            } while (!claim_.compare_exchange_weak(c, c + 1, std::memory_order_acq_rel, std::memory_order_acquire));
            try {
                (*job_)(i);
            } catch (...) {
                std::lock_guard<std::mutex> lk(m_);
                if (!err_) err_ = std::current_exception();
            }
            done_.fetch_add(1, std::memory_order_acq_rel);
        }
    }
    std::vector<std::thread> workers_;
    std::mutex busy_, m_;
    std::condition_variable cv_;
    std::function<void(int)>* job_ = nullptr;
    std::atomic<int> n_{0};
    unsigned long long pass_ = 0;
    std::atomic<unsigned long long> claim_{0};   // pass << 32 | next piece
    std::atomic<int> done_{0};
    std::atomic<bool> stop_{false};
    std::exception_ptr err_;
};

template <class F>
void par_for(int n, F f) {
    SetupPool& pool = SetupPool::get();
    if (n <= 1 || pool.size() <= 1 || !pool.run(n, f))
        for (int i = 0; i < n; ++i) f(i);
}

inline bool is_gp(int kind) { return kind == LBA_MONO_GP || kind == LBA_STEREO_GP; }
inline int obs_dim(int kind) { return (kind == LBA_STEREO_GP || kind == LBA_STEREO) ? 3 : 2; }

void normalize_q(const double* q, double* o) {
    const Quat n = qnormalize(Quat{q[0], q[1], q[2], q[3]});
    o[0] = n.x; o[1] = n.y; o[2] = n.z; o[3] = n.w;
}

// 6x6 inverse (Gauss-Jordan, partial pivoting) for GaussianProcess::mQcInv = Qc.inverse()
bool inverse6(const double* A, double* R) {
    double M[6][12];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 12; ++j) M[i][j] = j < 6 ? A[i * 6 + j] : (j - 6 == i ? 1.0 : 0.0);
    for (int c = 0; c < 6; ++c) {
        int piv = c;
        for (int r = c + 1; r < 6; ++r)
            if (std::fabs(M[r][c]) > std::fabs(M[piv][c])) piv = r;
        if (M[piv][c] == 0.0) return false;
        if (piv != c)
            for (int j = 0; j < 12; ++j) std::swap(M[c][j], M[piv][j]);
        const double d = M[c][c];
        for (int j = 0; j < 12; ++j) M[c][j] /= d;
        for (int r = 0; r < 6; ++r)
            if (r != c) {
                const double f = M[r][c];
                if (f != 0.0)
                    for (int j = 0; j < 12; ++j) M[r][j] -= f * M[c][j];
            }
    }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) R[i * 6 + j] = M[i][6 + j];
    return true;
}

// a device range of set_problem's to be zeroed by the set-up's single k_zero_ranges launch (flush_zero_ranges); the
// ranges are fresh buffers no upload of the set-up writes, so clearing them all at its end keeps the stream order
void zero_later(lba_problem* p, void* d, size_t bytes) {
    p->zero_list.push_back((unsigned long long)(uintptr_t)d);
    p->zero_list.push_back((bytes + 3) / 4);   // (every range is a whole number of 4-byte words)
}
void flush_zero_ranges(lba_problem* p);

inline int ublock_id(int n_pb, int bi, int bj) { return bi * n_pb - bi * (bi - 1) / 2 + (bj - bi); }

// ------------------------------------------------------------------------------------------------
// scratch array k of set_problem, n elements (contents unspecified: the caller writes every element)
std::vector<int>& scr_int(lba_problem* p, int k, size_t n) {
    p->scr_i[k].resize(n);
    return p->scr_i[k];
}
std::vector<double>& scr_dbl(lba_problem* p, int k, size_t n) {
    p->scr_d[k].resize(n);
    return p->scr_d[k];
}

int set_problem(lba_problem* p, const lba_kf* kfs, int n_kf, const double* lm_xyz, int n_lm, const lba_obs* obs,
                int n_obs, const lba_prior* priors, int n_priors, const int32_t* vel_kfs, int n_vel,
                const lba_cam* cams, int n_cam) {
    if (n_kf < 0 || n_lm < 0 || n_obs < 0 || n_priors < 0 || n_vel < 0 || n_cam < 0)
        throw ApiError{LBA_E_ARG, "negative array size"};
    if ((n_kf && !kfs) || (n_lm && !lm_xyz) || (n_obs && !obs) || (n_priors && !priors) || (n_vel && !vel_kfs) ||
        (n_cam && !cams))
        throw ApiError{LBA_E_ARG, "null array with non-zero size"};
    // the first invalid observation (pieces in parallel; the serial pass below names it).  The same pass counts each
    // piece's observations per landmark (the counting sort into observations by landmark, below) and marks the
    // keyframes the piece touches (activity): the caller's 64-byte records are read once for the three
    constexpr int VP = SETUP_PIECES;
    int first_bad = n_obs;
    const bool lm_hist = n_lm > 0 && (long long)n_lm * VP <= (8LL << 20);   // (else: the serial counting sort)
    std::vector<int>& lm_cnt = scr_int(p, 13, lm_hist ? (size_t)VP * n_lm : 0);
    std::vector<char> kf_mark((size_t)VP * std::max(n_kf, 1), 0);
    {
        int bad_at[VP];
        par_for(VP, [&](int piece) {
            const int i0 = (int)((long long)n_obs * piece / VP), i1 = (int)((long long)n_obs * (piece + 1) / VP);
            bad_at[piece] = n_obs;
            int* hc = lm_hist ? lm_cnt.data() + (size_t)piece * n_lm : nullptr;
            if (hc) std::fill(hc, hc + n_lm, 0);
            char* km = kf_mark.data() + (size_t)piece * std::max(n_kf, 1);
            for (int i = i0; i < i1; ++i) {
                const lba_obs& o = obs[i];
                bool ok = o.kind >= LBA_MONO_GP && o.kind <= LBA_STEREO && o.kf_b >= 0 && o.kf_b < n_kf && o.lm >= 0 &&
                          o.lm < n_lm && o.cam >= 0 && o.cam < n_cam && o.cam <= 255;
                if (ok && (o.kind == LBA_MONO_GP || o.kind == LBA_STEREO_GP))
                    ok = o.kf_a >= 0 && o.kf_a < n_kf && o.kf_a != o.kf_b &&
                         std::fabs(kfs[o.kf_b].time - kfs[o.kf_a].time) > 1e-6;
                if (!ok) { bad_at[piece] = i; break; }
                if (hc) ++hc[o.lm];
                km[o.kf_b] = 1;
                if (is_gp(o.kind)) km[o.kf_a] = 1;
            }
        });
        for (int piece = 0; piece < VP; ++piece) first_bad = std::min(first_bad, bad_at[piece]);
    }
    for (int i = first_bad; i < n_obs; ++i) {
        const lba_obs& o = obs[i];
        if (o.kind < LBA_MONO_GP || o.kind > LBA_STEREO) throw ApiError{LBA_E_ARG, "obs " + std::to_string(i) + ": bad kind"};
        if (o.kf_b < 0 || o.kf_b >= n_kf || o.lm < 0 || o.lm >= n_lm || o.cam < 0 || o.cam >= n_cam || o.cam > 255)
            throw ApiError{LBA_E_ARG, "obs " + std::to_string(i) + ": index out of range"};
        if (is_gp(o.kind)) {
            if (o.kf_a < 0 || o.kf_a >= n_kf || o.kf_a == o.kf_b)
                throw ApiError{LBA_E_ARG, "obs " + std::to_string(i) + ": bad kf_a"};
            if (!(std::fabs(kfs[o.kf_b].time - kfs[o.kf_a].time) > 1e-6))   // QiInv assert (GaussianProcess.h:32)
                throw ApiError{LBA_E_ARG, "obs " + std::to_string(i) + ": keyframe times too close"};
        }
    }
    for (int i = 0; i < n_priors; ++i) {
        const lba_prior& e = priors[i];
        if (e.kf_a < 0 || e.kf_a >= n_kf || e.kf_b < 0 || e.kf_b >= n_kf || e.kf_a == e.kf_b)
            throw ApiError{LBA_E_ARG, "prior " + std::to_string(i) + ": bad vertex"};
        if (!(std::fabs(kfs[e.kf_b].time - kfs[e.kf_a].time) > 1e-6))
            throw ApiError{LBA_E_ARG, "prior " + std::to_string(i) + ": keyframe times too close"};
    }
    for (int i = 0; i < n_vel; ++i)
        if (vel_kfs[i] < 0 || vel_kfs[i] >= n_kf) throw ApiError{LBA_E_ARG, "velocity edge: bad vertex"};
    std::vector<int> ext_cams;   // cameras with a free extrinsic, ascending (g2o vertex ids iniMPid + c + 1)
    for (int c = 0; c < n_cam; ++c)
        if (cams[c].ext_free) ext_cams.push_back(c);
    if (!ext_cams.empty()) {
        if (p->part_n > 0) throw ApiError{LBA_E_LIMIT, "free extrinsics are not supported in a partitioned problem"};
        for (int i = 0; i < n_obs; ++i)   // EdgeStereoGP projects through the static MultiKeyFrame::mTbc
            if (obs[i].kind == LBA_STEREO_GP && cams[obs[i].cam].ext_free)
                throw ApiError{LBA_E_ARG, "obs " + std::to_string(i) + ": stereo GP observation of a camera with a free extrinsic"};
    }

    // LBA_SETUP_TIMING: wall time of the set-up phases on stderr (host preprocessing vs device upload)
    const bool stime = std::getenv("LBA_SETUP_TIMING") != nullptr;
    auto tlast = std::chrono::steady_clock::now();
    p->setup_ms.clear();
    auto tsub = tlast;
    auto sub = [&](const char* what) {   // finer stamps inside a phase (LBA_SETUP_TIMING only)
        if (!stime) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "    %-22s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tsub).count());
        tsub = now;
    };
    auto mark = [&](const char* what) {
        if (p->stream) flush_uploads(p);   // (the arrays staged in this phase go out while the next one runs)
        const auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - tlast).count();
        p->setup_ms.push_back(ms);
        if (stime) std::fprintf(stderr, "set_problem %-12s %8.3f ms\n", what, ms);
        tlast = tsub = now;
    };
    p->status_entered = false;
    if (p->stream) HIPCHK(hipStreamSynchronize(p->stream));   // (the buffers are reused below)
    free_all(p);
    p->zero_list.clear();
    p->n_kf = n_kf; p->n_lm = n_lm; p->n_obs = n_obs; p->n_cam = n_cam;
    p->lm_host.assign(lm_xyz, lm_xyz + 3 * (size_t)n_lm);
    p->kf_fixed.resize(n_kf);
    for (int k = 0; k < n_kf; ++k) p->kf_fixed[k] = kfs[k].fixed != 0;

    // ---- active vertices (SparseOptimizer::initializeOptimization: a vertex is active if an edge
    //      that is not all-fixed touches it, sparse_optimizer.cpp:197-267)
    std::vector<char> kf_act(n_kf, 0), lm_act(n_lm, 0);
    for (int piece = 0; piece < VP; ++piece)
        for (int k = 0; k < n_kf; ++k) kf_act[k] |= kf_mark[(size_t)piece * std::max(n_kf, 1) + k];
    // observations by original landmark (stable): a counting sort, the counts from the validation pass
    std::vector<int> lo0(n_lm + 1, 0);
    std::vector<int>& lo_of = scr_int(p, 1, n_obs);
    if (lm_hist) {
        par_for(VP, [&](int piece) {   // per landmark: its total, and every piece's offset (its earlier pieces' counts)
            for (int l = (int)((long long)n_lm * piece / VP); l < (int)((long long)n_lm * (piece + 1) / VP); ++l) {
                int run = 0;
                for (int q = 0; q < VP; ++q) {
                    int& c = lm_cnt[(size_t)q * n_lm + l];
                    const int v = c;
                    c = run;
                    run += v;
                }
                lo0[l + 1] = run;
            }
        });
        for (int l = 0; l < n_lm; ++l) lo0[l + 1] += lo0[l];
        par_for(VP, [&](int piece) {
            int* off = lm_cnt.data() + (size_t)piece * n_lm;
            for (int i = (int)((long long)n_obs * piece / VP); i < (int)((long long)n_obs * (piece + 1) / VP); ++i) {
                const int l = obs[i].lm;
                lo_of[lo0[l] + off[l]++] = i;
            }
        });
    } else {
        for (int i = 0; i < n_obs; ++i) lo0[obs[i].lm + 1]++;
        for (int l = 0; l < n_lm; ++l) lo0[l + 1] += lo0[l];
        std::vector<int> fill(lo0.begin(), lo0.end() - 1);
        for (int i = 0; i < n_obs; ++i) lo_of[fill[obs[i].lm]++] = i;
    }
    for (int l = 0; l < n_lm; ++l) lm_act[l] = lo0[l + 1] > lo0[l];
    std::vector<lba_prior> pri;
    for (int i = 0; i < n_priors; ++i)
        if (!(kfs[priors[i].kf_a].fixed && kfs[priors[i].kf_b].fixed)) {
            pri.push_back(priors[i]);
            kf_act[priors[i].kf_a] = kf_act[priors[i].kf_b] = 1;
        }
    std::vector<int> vel;
    for (int i = 0; i < n_vel; ++i)
        if (!kfs[vel_kfs[i]].fixed) {
            vel.push_back(vel_kfs[i]);
            kf_act[vel_kfs[i]] = 1;
        }
    // partitioned: every rank carries every non-fixed keyframe (activity is the union over the ranks'
    // edges; the caller's global graph connects them all through the motion priors on rank 0)
    if (p->part_n > 0)
        for (int k = 0; k < n_kf; ++k)
            if (!kfs[k].fixed) kf_act[k] = 1;
    // free extrinsics (always active: their EdgeExtrinsicPrior is not all-fixed) as KF slots after the
    // keyframes, pose blocks after the keyframes' (g2o orders the active vertices by id)
    const int n_ext = (int)ext_cams.size(), n_kfs = n_kf + n_ext;
    std::vector<int> cam_slot(n_cam, -1);
    p->kf_hidx.assign(n_kfs, -1);
    int n_pb = 0;
    for (int k = 0; k < n_kf; ++k)
        if (kf_act[k] && !kfs[k].fixed) p->kf_hidx[k] = n_pb++;
    const int n_pb_kf = n_pb;
    for (int e = 0; e < n_ext; ++e) {
        cam_slot[ext_cams[e]] = n_kf + e;
        p->kf_hidx[n_kf + e] = n_pb++;
    }
    p->n_ext = n_ext;
    p->ext_cams = ext_cams;
    p->cams.assign(cams, cams + n_cam);
    p->n_pb = n_pb;
    p->np = 12 * n_pb;
    p->np_ext = 12 * n_pb_kf + 6 * n_ext;
    p->pose_ext.assign(p->np, -1);
    for (int i = 0; i < p->np; ++i)
        if (i < 12 * n_pb_kf) p->pose_ext[i] = i;
        else if (i % 12 < 6) p->pose_ext[i] = 12 * n_pb_kf + 6 * ((i - 12 * n_pb_kf) / 12) + i % 12;
    // the extrinsic block an observation links (EdgeMonoGPExtrinsic's vertex 3), or -1
    auto ext_block = [&](const lba_obs& o) { return o.kind == LBA_MONO_GP && cam_slot[o.cam] >= 0 ? p->kf_hidx[cam_slot[o.cam]] : -1; };
    if ((p->cfg.flags & LBA_FLAG_DENSE_SOLVE) && p->np > CF_DENSE_MAX_NP * CHOL_NB)
        throw ApiError{LBA_E_LIMIT, "the L^-1-tile solve is limited to pose systems of 6144"};
    const std::vector<int>& H = p->kf_hidx;

    sub("checks + activity");
    // GP (prev KF, KF) pairs, numbered in order of first appearance; gp_of: each GP observation's pair
    // (per KF b a short list of its pairs: (KF a, pair index); usually one, the previous keyframe)
    // (in parallel: every piece lists its distinct pairs in first-appearance order; the pieces' lists, merged in
    // piece order, give the pairs in first appearance over all observations; then every GP observation's pair)
    std::vector<std::vector<std::pair<int, int>>> gp_by_b(n_kf);
    std::vector<int> gp_a, gp_b, gp_of(n_obs, -1);
    {
        std::vector<std::vector<std::pair<int, int>>> first(VP);   // per piece: (kf_a, kf_b) in first-appearance order
        par_for(VP, [&](int piece) {
            std::vector<std::vector<int>> seen_a(n_kf);   // per KF b: the KFs a this piece has listed
            auto& out = first[piece];
            for (int i = (int)((long long)n_obs * piece / VP); i < (int)((long long)n_obs * (piece + 1) / VP); ++i) {
                const lba_obs& o = obs[i];
                if (!is_gp(o.kind)) continue;
                std::vector<int>& sa = seen_a[o.kf_b];
                if (std::find(sa.begin(), sa.end(), o.kf_a) != sa.end()) continue;
                sa.push_back(o.kf_a);
                out.emplace_back(o.kf_a, o.kf_b);
            }
        });
        for (int piece = 0; piece < VP; ++piece)
            for (const auto& ab : first[piece]) {
                auto& lst = gp_by_b[ab.second];
                bool have = false;
                for (const auto& e : lst)
                    if (e.first == ab.first) { have = true; break; }
                if (have) continue;
                lst.emplace_back(ab.first, (int)gp_a.size());
                gp_a.push_back(ab.first);
                gp_b.push_back(ab.second);
            }
        par_for(VP, [&](int piece) {
            for (int i = (int)((long long)n_obs * piece / VP); i < (int)((long long)n_obs * (piece + 1) / VP); ++i) {
                const lba_obs& o = obs[i];
                if (!is_gp(o.kind)) continue;
                for (const auto& e : gp_by_b[o.kf_b])
                    if (e.first == o.kf_a) { gp_of[i] = e.second; break; }
            }
        });
    }
    sub("  GP pair numbering");

    // GP pose samples: distinct observation times per GP pair (one per camera time stamp in
    // LocalGPBA), contiguous per pair; observations of a camera with a free extrinsic get samples of
    // their own (key: time, camera), so a sample couples at most one extrinsic block
    std::vector<int> gp_s0(gp_a.size() + 1, 0), sample_of(n_obs, -1), gps_cam;
    std::vector<double> gps_t;
    {
        typedef std::pair<double, int> SKey;
        auto skey = [&](const lba_obs& o) { return SKey(o.t, ext_block(o) >= 0 ? o.cam : -1); };
        // distinct keys per pair are few: each of 8 observation pieces keeps up to KC distinct keys per pair
        // inline (flat arrays), more in a per-piece overflow list; then per pair the union, sorted
        const int ng = (int)gp_a.size();
        constexpr int KC = 16, NPC = SETUP_PIECES;
        std::vector<SKey> pk((size_t)NPC * std::max(ng, 1) * KC);
        std::vector<int> pc((size_t)NPC * std::max(ng, 1), 0);
        std::vector<std::vector<std::pair<int, SKey>>> pov(NPC);
        par_for(NPC, [&](int piece) {
            SKey* K = pk.data() + (size_t)piece * ng * KC;
            int* C = pc.data() + (size_t)piece * ng;
            for (int i = (int)((long long)n_obs * piece / NPC); i < (int)((long long)n_obs * (piece + 1) / NPC); ++i)
                if (is_gp(obs[i].kind)) {
                    const int g = gp_of[i];
                    const SKey k = skey(obs[i]);
                    SKey* v = K + (size_t)g * KC;
                    bool seen = false;
                    for (int c = 0; c < C[g]; ++c)
                        if (v[c] == k) { seen = true; break; }
                    if (seen) continue;
                    if (C[g] < KC) v[C[g]++] = k;
                    else pov[piece].emplace_back(g, k);
                }
        });
        std::vector<std::vector<SKey>> ts(ng);
        for (int piece = 0; piece < NPC; ++piece) {
            const SKey* K = pk.data() + (size_t)piece * ng * KC;
            const int* C = pc.data() + (size_t)piece * ng;
            for (int g = 0; g < ng; ++g) ts[g].insert(ts[g].end(), K + (size_t)g * KC, K + (size_t)g * KC + C[g]);
            for (const auto& e : pov[piece]) ts[e.first].push_back(e.second);
        }
        sub("  GP sample keys");
        std::vector<SKey> keys;
        for (size_t g = 0; g < ts.size(); ++g) {
            std::sort(ts[g].begin(), ts[g].end());
            ts[g].erase(std::unique(ts[g].begin(), ts[g].end()), ts[g].end());
            gp_s0[g + 1] = gp_s0[g] + (int)ts[g].size();
            for (const SKey& k : ts[g]) { gps_t.push_back(k.first); gps_cam.push_back(k.second); keys.push_back(k); }
        }
        sub("  GP sample sort");
        par_for(SETUP_PIECES, [&](int piece) {
            for (int i = (int)((long long)n_obs * piece / SETUP_PIECES); i < (int)((long long)n_obs * (piece + 1) / SETUP_PIECES); ++i)
                if (is_gp(obs[i].kind)) {
                    const int g = gp_of[i];
                    const SKey* b = keys.data() + gp_s0[g];
                    sample_of[i] = gp_s0[g] + (int)(std::lower_bound(b, b + (gp_s0[g + 1] - gp_s0[g]), skey(obs[i])) - b);
                }
        });
    }

    sub("GP pairs + samples");
    // pose sample of every observation: its GP sample, or the KF pose record n_gps + kf_b
    const int n_gps = (int)gps_t.size(), n_smp = n_gps + n_kfs;
    std::vector<int>& smp_of = scr_int(p, 0, n_obs);
    par_for(VP, [&](int piece) {
        for (int i = (int)((long long)n_obs * piece / VP); i < (int)((long long)n_obs * (piece + 1) / VP); ++i)
            smp_of[i] = is_gp(obs[i].kind) ? sample_of[i] : n_gps + obs[i].kf_b;
    });

    // ---- heavy landmarks: a landmark whose observations / keyframes exceed one tile of k_lin_schur (a
    //      long track: LocalGPBA adds every observation of a local point, up to every keyframe of the
    //      window plus GP observations from non-keyframes, src/Optimizer.cc:1050-1200) is linearised in
    //      segment tiles and merged / eliminated by k_expand (heavy_item); heavy landmarks go last in
    //      device order.  tile_fits: the LDS limits of one k_lin_schur workgroup
    auto tile_fits = [&](int no, int nr, int npair, int nlmt, int nkf, int ns, int ne) {
        return no <= TILE_OBS && nr <= TILE_ROWS && npair <= TILE_PAIRS && nlmt <= TILE_LMS && nkf <= TILE_KF &&
               ns <= TILE_SMP && ne <= TILE_PROWS;
    };
    // per landmark: the span of non-fixed KFs observing it (device order key), heavy or not
    std::vector<int> lmin(n_lm, INT_MAX), lmax(n_lm, INT_MAX), lm_npl(n_lm, 0);
    std::vector<char> heavy(n_lm, 0);
    par_for(SETUP_PIECES, [&](int piece) {
        // distinct pose blocks / samples of a landmark counted by stamping (stamp = landmark + 1)
        std::vector<int> kst_((size_t)std::max(n_pb, 1), 0), sst_((size_t)std::max(n_gps + n_kfs, 1), 0);
        // (plain pointers and per-landmark locals: through the vectors every int store could alias every int
        // load, and the compiler reloaded the tables per observation)
        int* __restrict__ kst = kst_.data();
        int* __restrict__ sst = sst_.data();
        const int* __restrict__ Hh = H.data();
        const int* __restrict__ lo = lo_of.data();
        const int* __restrict__ lz = lo0.data();
        const int* __restrict__ so = smp_of.data();
        const int* __restrict__ cslot = cam_slot.data();
        for (int l = (int)((long long)n_lm * piece / SETUP_PIECES); l < (int)((long long)n_lm * (piece + 1) / SETUP_PIECES); ++l) {
            if (!lm_act[l]) continue;
            int nr = 0, ne = 0, npl = 0, ns = 0, mn = INT_MAX, mx = INT_MAX;
            const int stamp = l + 1;
            for (int q = lz[l]; q < lz[l + 1]; ++q) {
                const int oi = lo[q];
                const lba_obs& o = obs[oi];
                const int hb = Hh[o.kf_b], ha = is_gp(o.kind) ? Hh[o.kf_a] : -1;
                const int hx = (o.kind == LBA_MONO_GP && cslot[o.cam] >= 0) ? Hh[cslot[o.cam]] : -1;   // ext_block(o)
                for (int k : {hb, ha})
                    if (k >= 0) {
                        mn = mn == INT_MAX ? k : std::min(mn, k);
                        mx = mx == INT_MAX ? k : std::max(mx, k);
                    }
                for (int k : {hb, ha, hx})
                    if (k >= 0 && kst[k] != stamp) { kst[k] = stamp; ++npl; }
                ne += (hb >= 0) + (ha >= 0) + (hx >= 0);
                nr += obs_dim(o.kind);
                const int sm = so[oi];
                if (sst[sm] != stamp) { sst[sm] = stamp; ++ns; }
            }
            lmin[l] = mn;
            lmax[l] = mx;
            heavy[l] = !tile_fits(lz[l + 1] - lz[l], nr, npl, 1, npl, ns, ne);
            lm_npl[l] = npl;   // (its distinct pose blocks: its (KF, landmark) pairs below)
        }
    });
    sub("heavy classification");
    std::vector<int> order;
    int n_heavy_lm = 0;
    {   // stable order by (heavy, lmin, lmax) (INT_MAX = observed by fixed KFs only, after every block):
        // three stable counting passes (lmax, lmin, heavy) over the active landmarks in index order
        auto key = [&](int v) { return v == INT_MAX ? n_pb : v; };
        std::vector<int> a, b;
        a.reserve(n_lm);
        for (int l = 0; l < n_lm; ++l)
            if (lm_act[l]) { a.push_back(l); n_heavy_lm += heavy[l]; }
        b.resize(a.size());
        std::vector<int> cnt((size_t)std::max(n_pb + 2, 3));
        auto pass = [&](auto kf, int nk) {
            std::fill(cnt.begin(), cnt.begin() + nk + 1, 0);
            for (int l : a) cnt[kf(l) + 1]++;
            for (int k = 0; k < nk; ++k) cnt[k + 1] += cnt[k];
            for (int l : a) b[cnt[kf(l)]++] = l;
            a.swap(b);
        };
        pass([&](int l) { return key(lmax[l]); }, n_pb + 1);
        pass([&](int l) { return key(lmin[l]); }, n_pb + 1);
        pass([&](int l) { return (int)heavy[l]; }, 2);
        order.swap(a);
    }
    const int nl = (int)order.size(), n_reg = nl - n_heavy_lm;
    p->n_lm_dev = nl;
    p->lm_orig = order;
    p->lm_dev.assign(n_lm, -1);
    for (int d = 0; d < nl; ++d) p->lm_dev[order[d]] = d;

    sub("landmark order");
    // observations grouped by device landmark (stable)
    std::vector<int> lobs0(nl + 1, 0);
    std::vector<int>& obs_of = scr_int(p, 2, n_obs);
    for (int d = 0; d < nl; ++d) lobs0[d + 1] = lobs0[d] + (lo0[order[d] + 1] - lo0[order[d]]);
    par_for(SETUP_PIECES, [&](int piece) {
        for (int d = (int)((long long)nl * piece / SETUP_PIECES); d < (int)((long long)nl * (piece + 1) / SETUP_PIECES); ++d) {
            const int l = order[d];
            std::copy(lo_of.begin() + lo0[l], lo_of.begin() + lo0[l + 1], obs_of.begin() + lobs0[d]);
        }
    });

    sub("obs by landmark");
    // (KF, landmark) pairs, per device landmark, ascending pose block
    std::vector<int> lm_pair0(nl + 1, 0), pair_lm, pair_kf;
    auto lm_blocks = [&](int d, std::vector<int>& ks) {   // the landmark's pose blocks, ascending, distinct
        ks.clear();
        for (int q = lobs0[d]; q < lobs0[d + 1]; ++q) {
            const lba_obs& o = obs[obs_of[q]];
            if (H[o.kf_b] >= 0) ks.push_back(H[o.kf_b]);
            if (is_gp(o.kind) && H[o.kf_a] >= 0) ks.push_back(H[o.kf_a]);
            if (ext_block(o) >= 0) ks.push_back(ext_block(o));
        }
        std::sort(ks.begin(), ks.end());
        ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
    };
    // counts (the distinct pose blocks the heavy classification counted), then the pairs themselves
    for (int d = 0; d < nl; ++d) lm_pair0[d + 1] = lm_pair0[d] + lm_npl[order[d]];
    const int n_pairs = lm_pair0[nl];
    pair_lm.resize(n_pairs);
    pair_kf.resize(n_pairs);
    par_for(SETUP_PIECES, [&](int piece) {
        std::vector<int> ks;
        for (int d = (int)((long long)nl * piece / SETUP_PIECES); d < (int)((long long)nl * (piece + 1) / SETUP_PIECES); ++d) {
            lm_blocks(d, ks);
            for (size_t i = 0; i < ks.size(); ++i) { pair_lm[lm_pair0[d] + i] = d; pair_kf[lm_pair0[d] + i] = ks[i]; }
        }
    });
    // lm_kfs[d]: the landmark's pose blocks (ascending) = its pairs' blocks
    struct Span {
        const int* p; size_t n;
        const int* begin() const { return p; }
        const int* end() const { return p + n; }
        size_t size() const { return n; }
        int operator[](size_t i) const { return p[i]; }
    };
    auto lm_kfs_at = [&](int d) { return Span{pair_kf.data() + lm_pair0[d], (size_t)(lm_pair0[d + 1] - lm_pair0[d])}; };
    struct LmKfs {
        decltype(lm_kfs_at)& f;
        Span operator[](int d) const { return f(d); }
    } lm_kfs{lm_kfs_at};

    mark("order/pairs");
    // ---- tiles: consecutive regular landmarks under the limits of one k_lin_schur workgroup (tile_fits),
    //      then the segment tiles of the heavy landmarks
    std::vector<int> t_obs0, t_nobs, t_lm0, t_nlm, t_pair0, t_npair, t_smp0, t_nsmp, t_sent0, t_nsent, t_kf0, t_nkf;
    std::vector<int> tkf_list, tsm_smp, tsm_rows, sent_l1, sent_l2, sent_k1, sent_k2;
    std::vector<int> ob_row(n_obs, 0);
    std::vector<int> pair_r0(n_pairs + 1, 0), pair_rows, lm_r0(nl + 1, 0), lm_rows;
    std::vector<int> pair_lk(std::max(n_pairs, 1), 0);   // regular pairs: tile-local KF | tile-local landmark << 8
    // heavy landmarks: segments (landmark slots nl + s), segment pairs (pair slots n_pairs + c) and, per
    // canonical pair of a heavy landmark, the segment pairs that sum into it
    std::vector<int> hv_lm, hv_seg0(1, 0), hv_hp0(1, 0), hp_src0(1, 0), hp_src;
    int n_stiles = 0, n_seg = 0, n_segpairs = 0;
    {
        // per observation in device order, what the tiling reads (contiguous instead of through obs_of):
        // pose blocks of KF b / KF a / the extrinsic (-1: none or fixed), rows, pose sample
        std::vector<int>&dhb = scr_int(p, 3, n_obs), &dha = scr_int(p, 4, n_obs), &dhx = scr_int(p, 5, n_obs),
                         &ddim = scr_int(p, 6, n_obs), &dsmp = scr_int(p, 7, n_obs);
        par_for(SETUP_PIECES, [&](int piece) {
            for (int q = (int)((long long)n_obs * piece / SETUP_PIECES); q < (int)((long long)n_obs * (piece + 1) / SETUP_PIECES); ++q) {
                const lba_obs& ob = obs[obs_of[q]];
                dhb[q] = H[ob.kf_b];
                dha[q] = is_gp(ob.kind) ? H[ob.kf_a] : -1;
                dhx[q] = ext_block(ob);
                ddim[q] = obs_dim(ob.kind);
                dsmp[q] = smp_of[obs_of[q]];
            }
        });
        sub("tile inputs");
        std::vector<unsigned long long> tob;
        // LDS rows of a tile's observations [q0, q1) grouped by pose sample: every sample of the tile owns
        // one contiguous row run (stable by observation within a sample)
        auto emit_rows = [&](int q0, int q1) {
            tob.clear();
            for (int q = q0; q < q1; ++q) tob.push_back(((unsigned long long)(unsigned)dsmp[q] << 32) | (unsigned)q);
            std::sort(tob.begin(), tob.end());
            t_smp0.push_back((int)tsm_smp.size());
            int row = 0;
            for (size_t i = 0; i < tob.size();) {
                const int sm = (int)(tob[i] >> 32), r0 = row;
                size_t j = i;
                for (; j < tob.size() && (int)(tob[j] >> 32) == sm; ++j) {
                    const int q = (int)(tob[j] & 0xffffffffu);
                    ob_row[q] = row;
                    row += ddim[q];
                }
                tsm_smp.push_back(sm);
                tsm_rows.push_back(r0 | ((row - r0) << 16));
                i = j;
            }
            t_nsmp.push_back((int)tsm_smp.size() - t_smp0.back());
        };
        // entry list of the pair of KF block k over observations [q0, q1) (tile-local observation | side << 16)
        auto emit_pair_rows = [&](int k, int q0, int q1, int obase) {
            for (int o = q0; o < q1; ++o) {
                if (dhb[o] == k) pair_rows.push_back((o - obase) | (1 << 16));
                if (dha[o] == k) pair_rows.push_back(o - obase);
                if (dhx[o] == k) pair_rows.push_back((o - obase) | (2 << 16));
            }
        };
        // regular tiles: the landmarks [0, n_reg) in SETUP_PIECES contiguous pieces, each cut greedily into tiles
        // on its own thread (tiles never straddle a piece boundary, so the tiling is the same for any thread
        // count).  The tiles' lists depend only on their own landmarks: they are built in a second pass, in
        // parallel over runs of consecutive tiles, and concatenated with their offsets.  (A window below 256
        // landmarks per piece is one piece: its cut is serial, its lists -- most of the work -- are not.)
        struct TileOut {
            std::vector<int> t_obs0, t_nobs, t_lm0, t_nlm, t_pair0, t_npair, t_smp0, t_nsmp, t_sent0, t_nsent, t_kf0,
                t_nkf, tkf_list, tsm_smp, tsm_rows, sent_l1, sent_l2, sent_k1, sent_k2, pair_rows, lm_rows;
        };
        const int n_pieces = n_reg >= 256 * SETUP_PIECES ? SETUP_PIECES : 1;
#ifndef LBA_TILE_OBS_CAP
#define LBA_TILE_OBS_CAP TILE_OBS
#endif
        const int obs_cap = LBA_TILE_OBS_CAP;   // (a smaller cap: A/B builds only, scripts/exp_build.sh)
        // pass 1, the cut: the first landmark of every tile, per piece
        std::vector<std::vector<int>> cut(n_pieces);
        par_for(n_pieces, [&](int piece) {
            const int cap = obs_cap;
            const int d_end = (int)((long long)n_reg * (piece + 1) / n_pieces);
            int d = (int)((long long)n_reg * piece / n_pieces);
            // the tile's sample / KF sets grow by the landmark's new elements, found through membership
            // marks (1: in the tile, 2: new for the landmark being tried)
            std::vector<int> uni, usm, new_s, new_k;
            std::vector<char> kmark((size_t)std::max(n_pb, 1), 0), smark((size_t)std::max(n_smp, 1), 0);
            uni.reserve(TILE_PAIRS + 8);
            usm.reserve(TILE_SMP + 8);
            while (d < d_end) {
                int nobs = 0, rows = 0, npair = 0, nlmt = 0, nent = 0;
                uni.clear();
                usm.clear();
                int e = d;
                while (e < d_end) {
                    int no = lobs0[e + 1] - lobs0[e], nr = 0, ne = 0;
                    new_s.clear();
                    new_k.clear();
                    for (int q = lobs0[e]; q < lobs0[e + 1]; ++q) {
                        nr += ddim[q];
                        if (!smark[dsmp[q]]) { smark[dsmp[q]] = 2; new_s.push_back(dsmp[q]); }
                        ne += (dhb[q] >= 0) + (dha[q] >= 0) + (dhx[q] >= 0);
                    }
                    for (int k : lm_kfs[e])
                        if (!kmark[k]) { kmark[k] = 2; new_k.push_back(k); }
                    const int npl = lm_pair0[e + 1] - lm_pair0[e];
                    const bool fits = tile_fits(nobs + no, rows + nr, npair + npl, nlmt + 1,
                                                (int)(uni.size() + new_k.size()), (int)(usm.size() + new_s.size()),
                                                nent + ne) &&
                                      (nlmt == 0 || nobs + no <= cap);
                    for (int v : new_s) smark[v] = fits ? 1 : 0;
                    for (int k : new_k) kmark[k] = fits ? 1 : 0;
                    if (!fits) {
                        if (e == d)   // (the heavy classification above takes every landmark a tile cannot hold)
                            throw ApiError{LBA_E_LIMIT, "internal: landmark " + std::to_string(order[e]) + " does not fit a tile"};
                        break;
                    }
                    nobs += no; rows += nr; npair += npl; nlmt += 1; nent += ne;
                    usm.insert(usm.end(), new_s.begin(), new_s.end());
                    uni.insert(uni.end(), new_k.begin(), new_k.end());
                    ++e;
                }
                for (int v : usm) smark[v] = 0;
                for (int k : uni) kmark[k] = 0;
                cut[piece].push_back(d);
                d = e;
            }
        });
        std::vector<int> tl_d;   // tile t: landmarks [tl_d[t], tl_d[t + 1])
        for (const auto& c : cut) tl_d.insert(tl_d.end(), c.begin(), c.end());
        const int n_rt = (int)tl_d.size();
        tl_d.push_back(n_reg);
        // pass 2, the lists: n_runs runs of consecutive tiles
        const int n_runs = std::min(SETUP_PIECES, n_rt);
        auto run_t0 = [&](int r) { return (int)((long long)n_rt * r / n_runs); };
        std::vector<TileOut> outs(n_runs);
        par_for(n_runs, [&](int run) {
            TileOut& T = outs[run];
            const int ta = run_t0(run), tb = run_t0(run + 1);
            std::vector<int> uni, usm;
            std::vector<char> kmark((size_t)std::max(n_pb, 1), 0), smark((size_t)std::max(n_smp, 1), 0);
            std::vector<int> sloc_v((size_t)std::max(n_smp, 1), 0);   // sample -> its rank in the tile
            int* sloc = sloc_v.data();
            int srows[TILE_SMP + 1];
            uni.reserve(TILE_PAIRS + 8);
            usm.reserve(TILE_SMP + 8);
            {   // capacity for the run's share of the outputs (no regrowth while building)
                const int la = tl_d[ta], lb = tl_d[tb];
                const int no_p = lobs0[lb] - lobs0[la], np_p = lm_pair0[lb] - lm_pair0[la];
                const int nt_est = tb - ta + 1;
                T.pair_rows.reserve((size_t)np_p * 4 + 16);
                T.lm_rows.reserve((size_t)no_p * 3 + 16);
                T.tsm_smp.reserve((size_t)nt_est * TILE_SMP / 2);
                T.tsm_rows.reserve((size_t)nt_est * TILE_SMP / 2);
                T.sent_l1.reserve((size_t)nt_est * 48); T.sent_l2.reserve((size_t)nt_est * 48);
                T.sent_k1.reserve((size_t)nt_est * 48); T.sent_k2.reserve((size_t)nt_est * 48);
                T.tkf_list.reserve((size_t)nt_est * TILE_KF);
            }
            for (int t = ta; t < tb; ++t) {
                const int d = tl_d[t], e = tl_d[t + 1];
                const int nobs = lobs0[e] - lobs0[d], npair = lm_pair0[e] - lm_pair0[d], nlmt = e - d;
                // the tile's pose blocks (uni) and pose samples (usm), sorted
                uni.clear();
                usm.clear();
                for (int l = d; l < e; ++l) {
                    for (int q = lobs0[l]; q < lobs0[l + 1]; ++q)
                        if (!smark[dsmp[q]]) { smark[dsmp[q]] = 1; usm.push_back(dsmp[q]); }
                    for (int k : lm_kfs[l])
                        if (!kmark[k]) { kmark[k] = 1; uni.push_back(k); }
                }
                for (int v : usm) smark[v] = 0;
                for (int k : uni) kmark[k] = 0;
                std::sort(uni.begin(), uni.end());
                std::sort(usm.begin(), usm.end());
                for (size_t i = 0; i < usm.size(); ++i) sloc[usm[i]] = (int)i;
                T.t_obs0.push_back(lobs0[d]); T.t_nobs.push_back(nobs);
                T.t_lm0.push_back(d); T.t_nlm.push_back(nlmt);
                T.t_pair0.push_back(lm_pair0[d]); T.t_npair.push_back(npair);
                T.t_kf0.push_back((int)T.tkf_list.size()); T.t_nkf.push_back((int)uni.size());
                for (int k : uni) T.tkf_list.push_back(k);
                auto local = [&](int k) { return (int)(std::lower_bound(uni.begin(), uni.end(), k) - uni.begin()); };
                // LDS rows grouped by pose sample: every sample of the tile owns one contiguous row run, the
                // samples ascending, observations ascending within a sample (a counting pass over the
                // tile's sorted sample list)
                T.t_smp0.push_back((int)T.tsm_smp.size());
                {
                    const int ns = (int)usm.size();
                    std::fill(srows, srows + ns + 1, 0);
                    for (int q = lobs0[d]; q < lobs0[e]; ++q) srows[sloc[dsmp[q]] + 1] += ddim[q];
                    for (int i = 0; i < ns; ++i) srows[i + 1] += srows[i];
                    for (int i = 0; i < ns; ++i) {
                        T.tsm_smp.push_back(usm[i]);
                        T.tsm_rows.push_back(srows[i] | ((srows[i + 1] - srows[i]) << 16));
                    }
                    for (int q = lobs0[d]; q < lobs0[e]; ++q) {
                        const int i = sloc[dsmp[q]];
                        ob_row[q] = srows[i] | (i << 16);   // (+ the tile-local sample: k_update's back-substitution)
                        srows[i] += ddim[q];
                    }
                }
                T.t_nsmp.push_back((int)T.tsm_smp.size() - T.t_smp0.back());
                // entry lists per pair, row lists per landmark, the pairs' tile-local (KF, landmark);
                // pair_r0 / lm_r0 hold run-local offsets until the concatenation below
                for (int l = d; l < e; ++l) {
                    for (int q = lm_pair0[l]; q < lm_pair0[l + 1]; ++q) {
                        const int k = pair_kf[q];
                        for (int o = lobs0[l]; o < lobs0[l + 1]; ++o) {
                            if (dhb[o] == k) T.pair_rows.push_back((o - lobs0[d]) | (1 << 16));
                            if (dha[o] == k) T.pair_rows.push_back(o - lobs0[d]);
                            if (dhx[o] == k) T.pair_rows.push_back((o - lobs0[d]) | (2 << 16));
                        }
                        pair_r0[q + 1] = (int)T.pair_rows.size();
                        pair_lk[q] = local(k) | ((l - d) << 8);
                    }
                    for (int o = lobs0[l]; o < lobs0[l + 1]; ++o)
                        for (int r = 0; r < ddim[o]; ++r) T.lm_rows.push_back((ob_row[o] & 0xffff) + r);
                    lm_r0[l + 1] = (int)T.lm_rows.size();
                }
                // Schur entries: every (k1 <= k2) pose-block pair co-observed by a landmark of the tile, in
                // (k1, k2) order (k_lin_schur writes C's blocks of exactly these KF pairs)
                {
                    bool co[TILE_KF][TILE_KF] = {};
                    int lk[TILE_KF];
                    for (int l = d; l < e; ++l) {
                        const Span ks = lm_kfs[l];
                        for (size_t a = 0; a < ks.size(); ++a) lk[a] = local(ks[a]);
                        for (size_t a = 0; a < ks.size(); ++a)
                            for (size_t b = a; b < ks.size(); ++b) co[lk[a]][lk[b]] = true;
                    }
                    const int nu = (int)uni.size();
                    T.t_sent0.push_back((int)T.sent_l1.size());
                    int nen = 0;
                    // the diagonal entries (every tile KF has one) first: k_lin_schur gives them 6 tasks (their
                    // strictly lower 6 x 6 corner is never assembled), the others 8
                    for (int i = 0; i < nu; ++i) {
                        ++nen;
                        T.sent_l1.push_back(i); T.sent_l2.push_back(i);
                        T.sent_k1.push_back(uni[i]); T.sent_k2.push_back(uni[i]);
                    }
                    for (int i = 0; i < nu; ++i)
                        for (int j = i + 1; j < nu; ++j)
                            if (co[i][j]) {
                                ++nen;
                                T.sent_l1.push_back(i); T.sent_l2.push_back(j);
                                T.sent_k1.push_back(uni[i]); T.sent_k2.push_back(uni[j]);
                            }
                    T.t_nsent.push_back(nen);
                }
            }
        });
        // the runs' lists concatenated: every output's per-run offsets first, then the runs copied in parallel
        // (a serial element-wise concatenation cost most of the tiling's wall time on 16 threads)
        {
            std::vector<TileOut*> po(n_runs);
            for (int run = 0; run < n_runs; ++run) po[run] = &outs[run];
            struct Cat {
                std::vector<int>* dst;
                std::vector<int> TileOut::*src;
                int add;   // 0: values as they are; 1 / 2 / 3: + the run's offset into tsm_smp / sent_l1 / tkf_list
            };
            const Cat cats[] = {
                {&t_obs0, &TileOut::t_obs0, 0}, {&t_nobs, &TileOut::t_nobs, 0}, {&t_lm0, &TileOut::t_lm0, 0},
                {&t_nlm, &TileOut::t_nlm, 0}, {&t_pair0, &TileOut::t_pair0, 0}, {&t_npair, &TileOut::t_npair, 0},
                {&t_smp0, &TileOut::t_smp0, 1}, {&t_nsmp, &TileOut::t_nsmp, 0}, {&t_sent0, &TileOut::t_sent0, 2},
                {&t_nsent, &TileOut::t_nsent, 0}, {&t_kf0, &TileOut::t_kf0, 3}, {&t_nkf, &TileOut::t_nkf, 0},
                {&tkf_list, &TileOut::tkf_list, 0}, {&tsm_smp, &TileOut::tsm_smp, 0}, {&tsm_rows, &TileOut::tsm_rows, 0},
                {&sent_l1, &TileOut::sent_l1, 0}, {&sent_l2, &TileOut::sent_l2, 0}, {&sent_k1, &TileOut::sent_k1, 0},
                {&sent_k2, &TileOut::sent_k2, 0}, {&pair_rows, &TileOut::pair_rows, 0}, {&lm_rows, &TileOut::lm_rows, 0}};
            constexpr int NC = (int)(sizeof(cats) / sizeof(cats[0]));
            // off[c][run]: where the run's part of output c starts
            std::vector<std::vector<size_t>> off(NC, std::vector<size_t>(n_runs + 1, 0));
            for (int c = 0; c < NC; ++c) {
                for (int run = 0; run < n_runs; ++run)
                    off[c][run + 1] = off[c][run] + (po[run]->*(cats[c].src)).size();
                cats[c].dst->resize(off[c][n_runs]);
            }
            auto at = [&](std::vector<int> TileOut::*m) {   // index of an output in cats
                for (int c = 0; c < NC; ++c)
                    if (cats[c].src == m) return c;
                return -1;
            };
            const int c_smp = at(&TileOut::tsm_smp), c_sent = at(&TileOut::sent_l1), c_kf = at(&TileOut::tkf_list);
            const int c_pr = at(&TileOut::pair_rows), c_lr = at(&TileOut::lm_rows);
            par_for(n_runs, [&](int run) {
                const TileOut& T = *po[run];
                for (int c = 0; c < NC; ++c) {
                    const std::vector<int>& src = T.*(cats[c].src);
                    const int a = cats[c].add == 1 ? (int)off[c_smp][run] : cats[c].add == 2 ? (int)off[c_sent][run]
                                : cats[c].add == 3 ? (int)off[c_kf][run] : 0;
                    int* d = cats[c].dst->data() + off[c][run];
                    for (size_t k = 0; k < src.size(); ++k) d[k] = src[k] + a;
                }
                const int d0 = tl_d[run_t0(run)], d1 = tl_d[run_t0(run + 1)];
                const int o_pr = (int)off[c_pr][run], o_lr = (int)off[c_lr][run];
                for (int q = lm_pair0[d0]; q < lm_pair0[d1]; ++q) pair_r0[q + 1] += o_pr;
                for (int l = d0; l < d1; ++l) lm_r0[l + 1] += o_lr;
            });
        }
        n_stiles = (int)t_obs0.size();
        sub("regular tiles");
        // heavy landmarks: their canonical pairs and landmark slots get no rows of their own
        for (int q = lm_pair0[n_reg]; q < n_pairs; ++q) pair_r0[q + 1] = (int)pair_rows.size();
        for (int l = n_reg; l < nl; ++l) lm_r0[l + 1] = (int)lm_rows.size();
        // segments: runs of a heavy landmark's observations under the limits of k_lin_schur's phases 1-4
        // (no elimination: no KF-union limit; a segment's pairs are its distinct pose blocks)
        std::vector<int> uni, usm;
        std::vector<char> kmark((size_t)std::max(n_pb, 1), 0), smark((size_t)std::max(n_smp, 1), 0);
        for (int l = n_reg; l < nl; ++l) {
            hv_lm.push_back(l);
            const int cp0 = lm_pair0[l], ncp = lm_pair0[l + 1] - cp0;
            std::vector<std::vector<int>> src(ncp);
            int q0 = lobs0[l];
            while (q0 < lobs0[l + 1]) {
                int q1 = q0, nr = 0, ne = 0;
                usm.clear();
                uni.clear();
                while (q1 < lobs0[l + 1]) {
                    const int neq = (dhb[q1] >= 0) + (dha[q1] >= 0) + (dhx[q1] >= 0);
                    const int ns = (int)usm.size() + !smark[dsmp[q1]];
                    int nk = (int)uni.size();
                    for (int k : {dhb[q1], dha[q1], dhx[q1]})
                        if (k >= 0 && !kmark[k]) { kmark[k] = 2; ++nk; }
                    const bool fits = q1 - q0 + 1 <= TILE_OBS && nr + ddim[q1] <= TILE_ROWS && nk <= TILE_PAIRS &&
                                      ns <= TILE_SMP && ne + neq <= TILE_PROWS;
                    for (int k : {dhb[q1], dha[q1], dhx[q1]})
                        if (k >= 0 && kmark[k] == 2) {
                            kmark[k] = fits ? 1 : 0;
                            if (fits) uni.push_back(k);
                        }
                    if (!fits) break;
                    if (!smark[dsmp[q1]]) { smark[dsmp[q1]] = 1; usm.push_back(dsmp[q1]); }
                    nr += ddim[q1];
                    ne += neq;
                    ++q1;
                }
                for (int v : usm) smark[v] = 0;
                for (int k : uni) kmark[k] = 0;
                std::sort(uni.begin(), uni.end());
                const int s = n_seg++, sp0 = n_segpairs;
                t_obs0.push_back(q0); t_nobs.push_back(q1 - q0);
                t_lm0.push_back(nl + s); t_nlm.push_back(1);
                t_pair0.push_back(n_pairs + sp0); t_npair.push_back((int)uni.size());
                t_kf0.push_back((int)tkf_list.size()); t_nkf.push_back(0);
                t_sent0.push_back((int)sent_l1.size()); t_nsent.push_back(0);
                emit_rows(q0, q1);
                for (size_t c = 0; c < uni.size(); ++c) {
                    emit_pair_rows(uni[c], q0, q1, q0);
                    pair_r0.push_back((int)pair_rows.size());
                    const int* kb = pair_kf.data() + cp0;
                    src[std::lower_bound(kb, kb + ncp, uni[c]) - kb].push_back(n_pairs + sp0 + (int)c);
                }
                n_segpairs += (int)uni.size();
                for (int o = q0; o < q1; ++o)
                    for (int r = 0; r < ddim[o]; ++r) lm_rows.push_back(ob_row[o] + r);
                lm_r0.push_back((int)lm_rows.size());
                q0 = q1;
            }
            hv_seg0.push_back(n_seg);
            for (int j = 0; j < ncp; ++j) {
                for (int v : src[j]) hp_src.push_back(v);
                hp_src0.push_back((int)hp_src.size());
            }
            hv_hp0.push_back(hv_hp0.back() + ncp);
        }
    }
    const int n_tiles = (int)t_obs0.size();
    const int n_sent = (int)sent_l1.size();
    const int n_heavy = (int)hv_lm.size();

    mark("tiles");
    // ---- partial-sum slots, sorted by reduction target
    // (tile, sample) M / g partials: per sample, its tiles in tile order
    std::vector<int> mcnt(n_smp + 1, 0);
    for (int sm : tsm_smp) mcnt[sm]++;
    auto prefix = [](const std::vector<int>& c) {
        std::vector<int> s(c.size(), 0);
        for (size_t i = 1; i < c.size(); ++i) s[i] = s[i - 1] + c[i - 1];
        return s;
    };
    std::vector<int> ms0 = prefix(mcnt), mfill(ms0);
    std::vector<int> tsm_meta(2 * std::max(tsm_smp.size(), (size_t)1), 0);
    for (size_t i = 0; i < tsm_smp.size(); ++i) {
        tsm_meta[2 * i] = tsm_rows[i];
        tsm_meta[2 * i + 1] = mfill[tsm_smp[i]]++;
    }
    const int n_mslots = ms0[n_smp];
    // Hpp / b_p slab entries: pose samples (N^T M N: aa, ab, bb over their KFs a, b), then motion priors,
    // then velocity edges
    const int n_ublocks = n_pb * (n_pb + 1) / 2;
    std::vector<int> ub_i(n_ublocks), ub_j(n_ublocks);
    for (int bi = 0; bi < n_pb; ++bi)
        for (int bj = bi; bj < n_pb; ++bj) {
            const int id = ublock_id(n_pb, bi, bj);
            ub_i[id] = bi; ub_j[id] = bj;
        }
    // (a sample of a camera with a free extrinsic also couples its block e: ae, be, ee, b_e; then the
    // extrinsic priors on their blocks as "b")
    std::vector<int> ent_a, ent_b, ent_e, ent_cam;
    for (int sm = 0; sm < n_smp; ++sm) {
        ent_e.push_back(-1); ent_cam.push_back(-1);
        if (mcnt[sm] == 0) { ent_a.push_back(-1); ent_b.push_back(-1); continue; }   // unobserved
        if (sm < n_gps) {
            const int g = (int)(std::upper_bound(gp_s0.begin(), gp_s0.end(), sm) - gp_s0.begin()) - 1;
            ent_a.push_back(H[gp_a[g]]); ent_b.push_back(H[gp_b[g]]);
            if (gps_cam[sm] >= 0) { ent_e.back() = H[cam_slot[gps_cam[sm]]]; ent_cam.back() = gps_cam[sm]; }
        } else {
            ent_a.push_back(-1); ent_b.push_back(H[sm - n_gps]);
        }
    }
    for (auto& e : pri) { ent_a.push_back(H[e.kf_a]); ent_b.push_back(H[e.kf_b]); ent_e.push_back(-1); ent_cam.push_back(-1); }
    for (int k : vel) { ent_a.push_back(-1); ent_b.push_back(H[k]); ent_e.push_back(-1); ent_cam.push_back(-1); }
    for (int e = 0; e < n_ext; ++e) { ent_a.push_back(-1); ent_b.push_back(H[n_kf + e]); ent_e.push_back(-1); ent_cam.push_back(-1); }
    const int n_entries = (int)ent_a.size();
    std::vector<int> hcnt(n_ublocks + 1, 0), gcnt(n_pb + 1, 0);
    for (int en = 0; en < n_entries; ++en) {
        const int a = ent_a[en], b = ent_b[en], x = ent_e[en];
        if (a >= 0) { hcnt[ublock_id(n_pb, a, a)]++; gcnt[a]++; }
        if (b >= 0) { hcnt[ublock_id(n_pb, b, b)]++; gcnt[b]++; }
        if (a >= 0 && b >= 0) hcnt[ublock_id(n_pb, std::min(a, b), std::max(a, b))]++;
        if (x >= 0) {   // extrinsic blocks follow every KF block: (a, x), (b, x) are upper as they stand
            hcnt[ublock_id(n_pb, x, x)]++; gcnt[x]++;
            if (a >= 0) hcnt[ublock_id(n_pb, a, x)]++;
            if (b >= 0) hcnt[ublock_id(n_pb, b, x)]++;
        }
    }
    std::vector<int> hs0 = prefix(hcnt), gs0 = prefix(gcnt);
    std::vector<int> hfill(hs0), gfill(gs0);
    std::vector<int> seg_slot(SEG_STRIDE * (size_t)std::max(n_entries, 1), -1),
        seg_gslot(GSEG_STRIDE * (size_t)std::max(n_entries, 1), -1);
    for (int en = 0; en < n_entries; ++en) {
        const int a = ent_a[en], b = ent_b[en], x = ent_e[en];
        int* sl = seg_slot.data() + SEG_STRIDE * (size_t)en;
        int* gl = seg_gslot.data() + GSEG_STRIDE * (size_t)en;
        sl[3] = 0;
        if (a >= 0) { sl[0] = hfill[ublock_id(n_pb, a, a)]++; gl[0] = gfill[a]++; }
        if (a >= 0 && b >= 0) { sl[1] = hfill[ublock_id(n_pb, std::min(a, b), std::max(a, b))]++; sl[3] = a > b; }
        if (b >= 0) { sl[2] = hfill[ublock_id(n_pb, b, b)]++; gl[1] = gfill[b]++; }
        if (x >= 0) {
            if (a >= 0) sl[4] = hfill[ublock_id(n_pb, a, x)]++;
            if (b >= 0) sl[5] = hfill[ublock_id(n_pb, b, x)]++;
            sl[6] = hfill[ublock_id(n_pb, x, x)]++;
            sl[7] = ent_cam[en];
            gl[2] = gfill[x]++;
        }
    }
    // the pose sample that writes each Hpp / b_p slot (fused expansion + assembly; -1: an edge item)
    std::vector<int> hs_prod(std::max(hs0[n_ublocks], 1), -1), gs_prod(std::max(gs0[n_pb], 1), -1);
    for (int en = 0; en < n_smp; ++en) {
        const int* sl = seg_slot.data() + SEG_STRIDE * (size_t)en;
        const int* gl = seg_gslot.data() + GSEG_STRIDE * (size_t)en;
        for (int q : {0, 1, 2, 4, 5, 6})
            if (sl[q] >= 0) hs_prod[sl[q]] = en;
        for (int q = 0; q < 3; ++q)
            if (gl[q] >= 0) gs_prod[gl[q]] = en;
    }
    // Schur partial blocks per (tile, KF pair) and rhs partials per (tile, KF)
    std::vector<int> scnt(n_ublocks + 1, 0), gpcnt(n_pb + 1, 0);
    for (int s = 0; s < n_sent; ++s) scnt[ublock_id(n_pb, sent_k1[s], sent_k2[s])]++;
    for (int k : tkf_list) gpcnt[k]++;
    for (int h = 0; h < n_heavy; ++h) {   // a heavy landmark: every pair (a <= b) of its KFs, every KF
        const Span ks = lm_kfs[hv_lm[h]];
        for (size_t a = 0; a < ks.size(); ++a) {
            gpcnt[ks[a]]++;
            for (size_t b = a; b < ks.size(); ++b) scnt[ublock_id(n_pb, ks[a], ks[b])]++;
        }
    }
    std::vector<int> ss0 = prefix(scnt), gps0 = prefix(gpcnt);
    std::vector<int> sfill(ss0), gpfill(gps0);
    std::vector<int> sslot(std::max(n_sent, 1)), tkf_gslot(std::max((int)tkf_list.size(), 1));
    for (int s = 0; s < n_sent; ++s) sslot[s] = sfill[ublock_id(n_pb, sent_k1[s], sent_k2[s])]++;
    for (size_t t = 0; t < tkf_list.size(); ++t) tkf_gslot[t] = gpfill[tkf_list[t]]++;
    std::vector<int> hv_ss0(1, 0), hv_sslot, hp_gslot;   // (after the regular tiles' slots of each target)
    for (int h = 0; h < n_heavy; ++h) {
        const Span ks = lm_kfs[hv_lm[h]];
        for (size_t a = 0; a < ks.size(); ++a) {
            hp_gslot.push_back(gpfill[ks[a]]++);
            for (size_t b = a; b < ks.size(); ++b) hv_sslot.push_back(sfill[ublock_id(n_pb, ks[a], ks[b])]++);
        }
        hv_ss0.push_back((int)hv_sslot.size());
    }
    const int n_hslots = hs0[n_ublocks], n_gslots = gs0[n_pb], n_sslots = ss0[n_ublocks], n_gpslots = gps0[n_pb];
    sub("slab slots");


    // ---- observations in device order
    std::vector<int>&ob_meta = scr_int(p, 8, n_obs), &ob_kfa = scr_int(p, 9, n_obs), &ob_kfb = scr_int(p, 10, n_obs),
                     &ob_smp = scr_int(p, 11, n_obs), &ob_lm = scr_int(p, 12, n_obs);
    std::vector<double>&ob_z = scr_dbl(p, 0, 3 * (size_t)n_obs), &ob_w = scr_dbl(p, 1, n_obs);
    p->obs_dev.assign(n_obs, -1);
    par_for(SETUP_PIECES, [&](int piece) {
    for (int q = (int)((long long)n_obs * piece / SETUP_PIECES); q < (int)((long long)n_obs * (piece + 1) / SETUP_PIECES); ++q) {
        const lba_obs& o = obs[obs_of[q]];
        p->obs_dev[obs_of[q]] = q;
        ob_meta[q] = o.kind | (o.cam << 4);
        ob_kfa[q] = is_gp(o.kind) ? o.kf_a : -1;
        ob_kfb[q] = o.kf_b;
        ob_smp[q] = smp_of[obs_of[q]];
        ob_lm[q] = p->lm_dev[o.lm];
        ob_z[3 * (size_t)q] = o.z[0]; ob_z[3 * (size_t)q + 1] = o.z[1]; ob_z[3 * (size_t)q + 2] = o.z[2];
        ob_w[q] = o.w;
    }
    });
    sub("device-order observations");
    // cameras: Tcb = Tbc^-1 as matrix (MultiKeyFrame::mTbc[c].cast<double>() normalises) and the
    // extrinsic factor Ad(Tbc) (lba::cam_record)
    std::vector<double> camd(CAMD_STRIDE * (size_t)std::max(n_cam, 1), 0.0);
    auto cam_se3 = [&](int c) {
        SE3 T;
        double q[4];
        normalize_q(cams[c].q, q);
        T.q = Quat{q[0], q[1], q[2], q[3]};
        for (int i = 0; i < 3; ++i) T.t[i] = cams[c].t[i];
        return T;
    };
    for (int c = 0; c < n_cam; ++c)
        cam_record(cam_se3(c), cams[c].fx, cams[c].fy, cams[c].cx, cams[c].cy, camd.data() + CAMD_STRIDE * c);
    // keyframe / landmark state (then the free extrinsics: Tbc as the pose, no velocity)
    std::vector<double> kst(KF_STRIDE * (size_t)std::max(n_kfs, 1), 0.0), lst(3 * (size_t)std::max(nl, 1), 0.0);
    for (int k = 0; k < n_kf; ++k) {
        double* o = kst.data() + KF_STRIDE * k;
        normalize_q(kfs[k].q, o);
        for (int i = 0; i < 3; ++i) o[4 + i] = kfs[k].t[i];
        for (int i = 0; i < 6; ++i) o[7 + i] = kfs[k].vel[i];
        o[13] = kfs[k].time;
        o[14] = kfs[k].bf;
    }
    std::vector<int> kf_cam(std::max(n_kfs, 1), -1), ep_kf(std::max(n_ext, 1), 0);
    std::vector<double> ep_data(16 * (size_t)std::max(n_ext, 1), 0.0);
    for (int e = 0; e < n_ext; ++e) {
        const int c = ext_cams[e];
        const SE3 T = cam_se3(c);
        double* o = kst.data() + KF_STRIDE * (size_t)(n_kf + e);
        o[0] = T.q.x; o[1] = T.q.y; o[2] = T.q.z; o[3] = T.q.w;
        for (int i = 0; i < 3; ++i) o[4 + i] = T.t[i];
        kf_cam[n_kf + e] = c;
        ep_kf[e] = n_kf + e;
        // EdgeExtrinsicPrior(R): R_ = R.inverse() of the widened, normalised mRbc_ini (so3.hpp:229-231)
        double qi[4];
        normalize_q(cams[c].rbc_ini, qi);
        const Quat ri = qinv(Quat{qi[0], qi[1], qi[2], qi[3]});
        double* d = ep_data.data() + 16 * (size_t)e;
        d[0] = ri.x; d[1] = ri.y; d[2] = ri.z; d[3] = ri.w;
        for (int i = 0; i < 9; ++i) d[4 + i] = cams[c].rbc_info[i];
    }
    for (int d = 0; d < nl; ++d)
        for (int i = 0; i < 3; ++i) lst[3 * (size_t)d + i] = lm_xyz[3 * (size_t)order[d] + i];
    std::vector<int> pri_a, pri_b;
    for (auto& e : pri) { pri_a.push_back(e.kf_a); pri_b.push_back(e.kf_b); }

    mark("slots/state");
    if (p->host_only) {   // (lba_setup_host_profile) a fingerprint of the tiling and the slab layout
        uint32_t h = 2166136261u;
        auto mix = [&](const std::vector<int>& v) {
            for (int x : v) { h ^= (uint32_t)x; h *= 16777619u; }
        };
        mix(t_obs0); mix(t_lm0); mix(tsm_meta); mix(pair_rows); mix(lm_rows); mix(pair_lk); mix(sent_l1); mix(sent_l2);
        mix(sslot); mix(tkf_gslot); mix(seg_slot); mix(ob_row);
        mix(t_nobs); mix(t_nlm); mix(t_pair0); mix(t_npair); mix(t_smp0); mix(t_nsmp); mix(t_sent0); mix(t_nsent);
        mix(t_kf0); mix(t_nkf); mix(tkf_list); mix(sent_k1); mix(sent_k2); mix(pair_r0); mix(lm_r0);
        p->setup_hash = h;
        p->setup_tiles = n_tiles;
        return LBA_OK;
    }
    // ---- device upload
    DevProblem& D = p->D;
    D.n_kf = n_kfs; D.n_kf_user = n_kf; D.n_eprior = n_ext; D.n_lm = nl; D.n_obs = n_obs; D.n_gp = (int)gp_a.size(); D.n_pairs = n_pairs;
    D.n_tiles = n_tiles; D.n_pb = n_pb; D.np = p->np; D.n_prior = (int)pri.size(); D.n_vel = (int)vel.size();
    D.n_cam = n_cam; D.n_entries = n_entries; D.n_sentries = n_sent; D.n_ublocks = n_ublocks;
    D.ob_meta = dupload(p, ob_meta); D.ob_kfa = dupload(p, ob_kfa); D.ob_kfb = dupload(p, ob_kfb);
    D.ob_smp = dupload(p, ob_smp); D.ob_lm = dupload(p, ob_lm);
    D.ob_row = dupload(p, ob_row);
    D.ob_z = dupload(p, ob_z); D.ob_w = dupload(p, ob_w);
    D.gp_s0 = dupload(p, gp_s0); D.gps_t = dupload(p, gps_t); D.n_gps = n_gps; D.n_smp = n_smp;
    D.kf_hidx = dupload(p, p->kf_hidx); D.gp_kfa = dupload(p, gp_a); D.gp_kfb = dupload(p, gp_b);
    {   // per GP pair: KF a, KF b and their pose blocks (k_update's trial states: one load, no kf_hidx hop)
        std::vector<int> hab(4 * std::max(gp_a.size(), (size_t)1), -1);
        for (size_t g = 0; g < gp_a.size(); ++g) {
            hab[4 * g] = gp_a[g];
            hab[4 * g + 1] = gp_b[g];
            hab[4 * g + 2] = p->kf_hidx[gp_a[g]];
            hab[4 * g + 3] = p->kf_hidx[gp_b[g]];
        }
        D.gp_hab = dupload(p, hab);
    }
    D.camdb[0] = dupload(p, camd);
    D.camdb[1] = dupload(p, camd);
    D.kf_cam = dupload(p, kf_cam);
    D.ep_kf = dupload(p, ep_kf);
    D.ep_data = dupload(p, ep_data);
    D.tile_obs0 = dupload(p, t_obs0); D.tile_nobs = dupload(p, t_nobs); D.tile_lm0 = dupload(p, t_lm0);
    D.tile_nlm = dupload(p, t_nlm); D.tile_pair0 = dupload(p, t_pair0); D.tile_npair = dupload(p, t_npair);
    D.tile_smp0 = dupload(p, t_smp0); D.tile_nsmp = dupload(p, t_nsmp); D.tsm_meta = dupload(p, tsm_meta);
    D.ms0 = dupload(p, ms0); D.tile_sent0 = dupload(p, t_sent0);
    D.tile_nsent = dupload(p, t_nsent); D.tile_kf0 = dupload(p, t_kf0); D.tile_nkf = dupload(p, t_nkf);
    D.tkf_list = dupload(p, tkf_list);
    {   // k_lin_schur's workgroup -> tile map: longest first by a cost estimate (list scheduling: the tiles
        // outnumber the resident workgroup slots, ~1.4x at config 1, and the costly tiles, many KFs and Schur
        // entries, sit at the end of the landmark order, so in index order the last round of workgroups ran
        // long after most CUs were idle).  Cost: a non-negative least-squares fit of measured tile durations
        // on the tile shape (us ~ 0.027 npair + 0.775 nlm + 0.077 nsent + 1.807 nkf, profiles/r3aq_tile_order.txt)
        std::vector<long long> cost(n_tiles);
        std::vector<int> perm(n_tiles);
        for (int t = 0; t < n_tiles; ++t) {
            cost[t] = 27LL * t_npair[t] + 775LL * t_nlm[t] + 77LL * t_nsent[t] + 1807LL * t_nkf[t];
            perm[t] = t;
        }
        // (LBA_DISPATCH_INDEX_ORDER: index order, for the tests that check the order changes no result)
        if (!std::getenv("LBA_DISPATCH_INDEX_ORDER"))
            std::stable_sort(perm.begin(), perm.end(), [&](int x, int y) { return cost[x] > cost[y]; });
        D.tile_perm = dupload(p, perm);
    }
    D.n_stiles = n_stiles; D.n_heavy = n_heavy;
    D.hv_lm = dupload(p, hv_lm); D.hv_seg0 = dupload(p, hv_seg0); D.hv_hp0 = dupload(p, hv_hp0);
    D.hp_src0 = dupload(p, hp_src0); D.hp_src = dupload(p, hp_src); D.hp_gslot = dupload(p, hp_gslot);
    D.hv_ss0 = dupload(p, hv_ss0); D.hv_sslot = dupload(p, hv_sslot);
    D.Vh = dalloc<double>(p, (size_t)36 * std::max(hv_hp0.back(), 1));
    D.pair_lk = dupload(p, pair_lk);
    D.sent_l1 = dupload(p, sent_l1); D.sent_l2 = dupload(p, sent_l2);
    D.pair_lm = dupload(p, pair_lm); D.pair_kf = dupload(p, pair_kf); D.pair_r0 = dupload(p, pair_r0);
    D.pair_rows = dupload(p, pair_rows); D.lm_r0 = dupload(p, lm_r0); D.lm_rows = dupload(p, lm_rows);
    D.lm_pair0 = dupload(p, lm_pair0);
    {   // k_update's sample-space back-substitution of the regular tiles' landmarks
        // per tile sample (tile order, beside tsm_smp): its sample's pose blocks and extrinsic camera
        std::vector<int> tsm_blk(4 * std::max(tsm_smp.size(), (size_t)1), -1);
        for (size_t j = 0; j < tsm_smp.size(); ++j) {
            const int sm = tsm_smp[j];
            tsm_blk[4 * j] = ent_a[sm];
            tsm_blk[4 * j + 1] = ent_b[sm];
            tsm_blk[4 * j + 2] = ent_e[sm];
            tsm_blk[4 * j + 3] = ent_cam[sm];
        }
        D.tsm_smp = dupload(p, tsm_smp);
        D.tsm_blk = dupload(p, tsm_blk);
        D.lm_obs0 = dupload(p, lobs0);
    }
    D.hfin = p->d_hfin;
    D.hlog = p->d_hlog;
    if (std::getenv("LBA_PHASE_TIMING")) {
        D.tdbg_lin = dalloc<unsigned long long>(p, (size_t)n_tiles * 16);
        D.tdbg_schur = dalloc<unsigned long long>(p, (size_t)n_tiles * 16);
        HIPCHK(hipMemsetAsync(D.tdbg_lin, 0, (size_t)n_tiles * 16 * 8, p->stream));
        HIPCHK(hipMemsetAsync(D.tdbg_schur, 0, (size_t)n_tiles * 16 * 8, p->stream));
        const int nblk = (p->np + CHOL_NB - 1) / CHOL_NB + 1;
        D.tdbg_chol = dalloc<unsigned long long>(p, (size_t)nblk * 16);
        D.tdbg_bs = dalloc<unsigned long long>(p, (size_t)nblk * 16);
        D.tdbg_cf = dalloc<unsigned long long>(p, (size_t)4096 * CF_TDBG_STRIDE);
        HIPCHK(hipMemsetAsync(D.tdbg_cf, 0, (size_t)4096 * CF_TDBG_STRIDE * 8, p->stream));
        HIPCHK(hipMemsetAsync(D.tdbg_chol, 0, (size_t)nblk * 16 * 8, p->stream));
        HIPCHK(hipMemsetAsync(D.tdbg_bs, 0, (size_t)nblk * 16 * 8, p->stream));
    }
    D.seg_slot = dupload(p, seg_slot); D.seg_gslot = dupload(p, seg_gslot);

    D.hs0 = dupload(p, hs0); D.gs0 = dupload(p, gs0); D.ub_i = dupload(p, ub_i); D.ub_j = dupload(p, ub_j);
    D.sslot = dupload(p, sslot); D.ss0 = dupload(p, ss0); D.tkf_gslot = dupload(p, tkf_gslot);
    D.gps0 = dupload(p, gps0);
    D.pri_a = dupload(p, pri_a); D.pri_b = dupload(p, pri_b); D.vel_kf = dupload(p, vel);
    D.pri_entry0 = n_smp;
    double qcinv[36];
    if (!inverse6(p->cfg.qc, qcinv)) throw ApiError{LBA_E_ARG, "Qc is singular"};
    for (int i = 0; i < 36; ++i) D.qcinv[i] = qcinv[i];
    D.huber_mono = p->cfg.huber_mono;
    D.huber_stereo = p->cfg.huber_stereo;
    D.huber_prior = p->cfg.huber_prior;
    {   // pose samples; the KF records' factor N = [0 | I 0] is constant (k_gp_prep writes their poses)
        std::vector<double> g0((size_t)GPS_STRIDE * std::max(n_smp, 1), 0.0);
        for (int k = 0; k < n_kfs; ++k)
            for (int l = 0; l < 6; ++l) g0[(size_t)(n_gps + k) * GPS_STRIDE + 12 + 6 * (12 + l) + l] = 1.0;
        D.gpsb[0] = dupload(p, g0);
        D.gpsb[1] = dupload(p, g0);
    }
    D.mslab = dalloc<double>(p, (size_t)MS_PITCH * std::max(n_mslots, 1));
    D.kfp_pose = dalloc<double>(p, (size_t)KFP_STRIDE * std::max(n_kfs, 1));
    D.hslab = dalloc<double>(p, (size_t)144 * std::max(n_hslots, 1));
    D.gslab = dalloc<double>(p, (size_t)GS_PITCH * std::max(n_gslots, 1));
    D.sslab = dalloc<double>(p, (size_t)144 * std::max(n_sslots, 1));
    D.gpslab = dalloc<double>(p, (size_t)GS_PITCH * std::max(n_gpslots, 1));
    D.n_mslots = n_mslots; D.n_hslots = n_hslots; D.n_gslots = n_gslots; D.n_sslots = n_sslots; D.n_gpslots = n_gpslots;
    const int npad = (p->np + CHOL_NB - 1) / CHOL_NB * CHOL_NB;
    mark("upload");
    // ---- solve layout of the reduced camera system: dissection order, tile structure of L, task lists
    {
        const int NP = npad / CHOL_NB;
        // natural tile pattern of S at panel granularity (structural blocks, diagonal), then the nested-
        // dissection order and the symbolic factorisation (lba_plan.hpp).  Panels holding rows of free
        // extrinsics (dense: they couple every keyframe) are ordered last.  A partition plans the union
        // pattern of its ranks' systems.
        const int NPk = std::min(NP, 12 * n_pb_kf / CHOL_NB + (n_ext ? 0 : NP));
        std::vector<std::vector<int>> lower(NP);
        for (int P = 0; P < NP; ++P) lower[P].push_back(P);
        std::vector<std::pair<int, int>> edge_panels;   // (this rank's edges' couplings: the split's check)
        auto couple = [&](int r, int c) {   // natural rows r, c of S
            const int P = std::max(r, c) / CHOL_NB, Q = std::min(r, c) / CHOL_NB;
            lower[P].push_back(Q);
            edge_panels.emplace_back(P, Q);
        };
        for (int u = 0; u < n_ublocks; ++u) {
            if (!(hcnt[u] > 0 || scnt[u] > 0)) continue;
            const int r0 = 12 * ub_j[u], c0 = 12 * ub_i[u];
            couple(r0, c0); couple(r0 + 11, c0); couple(r0, c0 + 11); couple(r0 + 11, c0 + 11);
        }
        for (int P = 0; P < NP; ++P) {
            std::sort(lower[P].begin(), lower[P].end());
            lower[P].erase(std::unique(lower[P].begin(), lower[P].end()), lower[P].end());
        }
        if (p->part_n > 0) part_status(p, 0);   // (every rank's preprocessing succeeded, or all throw)
        if (p->part_n > 0) {   // the union pattern of the ranks' systems (one all-reduce, at set-up)
            std::vector<double> occ((size_t)NP * NP, 0.0);
            for (int P = 0; P < NP; ++P)
                for (int Q : lower[P]) occ[(size_t)P * NP + Q] = 1.0;
            double* d = dalloc<double>(p, occ.size());
            HIPCHK(hipMemcpy(d, occ.data(), occ.size() * sizeof(double), hipMemcpyHostToDevice));
            preduce(p, d, (int64_t)occ.size());
            HIPCHK(hipStreamSynchronize(p->stream));
            HIPCHK(hipMemcpy(occ.data(), d, occ.size() * sizeof(double), hipMemcpyDeviceToHost));
            for (int P = 0; P < NP; ++P) {
                lower[P].clear();
                for (int Q = 0; Q <= P; ++Q)
                    if (occ[(size_t)P * NP + Q] != 0.0 || Q == P) lower[P].push_back(Q);
            }
        }
        sub("  S pattern");
        const lba_plan::Plan& pl = plan_panels_cached(p->plan_cache, NP, NPk, lower);
        sub("  dissection plan");
        p->chain = pl.chain;
        p->nd_tail = pl.tail;
        p->nd_levels = pl.levels;
        // distributed factorisation (LBA_FLAG_SUBTREE_SOLVE, partitioned problems): the elimination tree cut into
        // one subtree per rank plus the top (lba_plan::split_subtrees, the same on every rank); this rank's
        // couplings must lie in its subtree and the top (lba_partition_assign gives such a landmark split)
        const bool split = p->part_n > 0 && (p->cfg.flags & LBA_FLAG_SUBTREE_SOLVE);
        const std::vector<int> own = split ? lba_plan::split_subtrees(pl, p->part_n) : std::vector<int>(NP, -1);
        if (split) {   // (a second status point: a rank whose couplings leave its subtree releases its peers)
            bool stray = false;
            for (const auto& e : edge_panels) {
                const int a = own[pl.ppos[e.first]], b = own[pl.ppos[e.second]];
                if ((a >= 0 && a != p->part_rank) || (b >= 0 && b != p->part_rank)) stray = true;
            }
            part_status(p, stray ? 1 : 0);
            if (stray)
                throw ApiError{LBA_E_ARG, "partitioned problem: a landmark or edge of rank " +
                                              std::to_string(p->part_rank) + " couples keyframes of another rank's "
                                              "subtree (split the window with lba_partition_assign)"};
        }
        p->split_own = own;
        p->ppos_h = pl.ppos;
        {   // the factorisation work this rank does: its subtree's columns and the top (split), or all of them
            const double b3 = (double)CHOL_NB * CHOL_NB * CHOL_NB;
            double f = 0.0;
            int n_own = 0, n_top = 0;
            for (int j = 0; j < NP; ++j) {
                if (own[j] >= 0 && own[j] != p->part_rank) continue;
                (own[j] < 0 ? n_top : n_own)++;
                const double m = (double)pl.colrows[j].size();
                f += b3 / 3.0 + m * b3 + m * b3 + m * (m - 1.0) * b3;
            }
            p->flops_factor_rank = f;
            p->split_panels[0] = split ? n_own : 0;
            p->split_panels[1] = split ? n_top : NP;
        }
        p->s_tiles = 0;
        for (int P = 0; P < NP; ++P) p->s_tiles += (int)lower[P].size();
        {   // per column with m tiles below the diagonal: potrf 32^3/3, m trsm 32^3, the m(m+1)/2 tile updates
            // of the trailing matrix (syrk 32^3 on the diagonal ones, gemm 2 x 32^3 below)
            const double b3 = (double)CHOL_NB * CHOL_NB * CHOL_NB;
            double f = 0.0;
            for (int j = 0; j < NP; ++j) {
                const double m = (double)pl.colrows[j].size();
                f += b3 / 3.0 + m * b3 + m * b3 + m * (m - 1.0) * b3;
            }
            p->flops_factor = f;
        }
        const std::vector<int>& ppos = pl.ppos;
        const std::vector<int>& pnat = pl.pnat;
        // rows: natural -> factorisation order, and back
        std::vector<int> rpos(npad), rnat(npad);
        for (int r = 0; r < npad; ++r) {
            rpos[r] = ppos[r / CHOL_NB] * CHOL_NB + r % CHOL_NB;
            rnat[rpos[r]] = r;
        }
        // solve path: L^-1 tiles (the solve has no substitution chain, but L^-1 is dense below the
        // diagonal: O(n^3) work) up to CF_AUTO_BAND_NP panels, substitution tasks above (or when asked)
        const bool band = split || (!(p->cfg.flags & LBA_FLAG_DENSE_SOLVE) &&
                                    ((p->cfg.flags & LBA_FLAG_BAND_SOLVE) || NP > CF_AUTO_BAND_NP));
        D.cf_band = band ? 1 : 0;
        const int ntile = pl.ntile();
        // dataflow factorisation + solve (k_chol_flow), tasks in topological order: per column c the
        // factor tiles of its rows (the diagonal first), then (L^-1 solve) the L^-1 tiles of row c; at the
        // end one solution task per panel.  Task t: (j, i, kind) with five tile ids (task_t) and a list of
        // update / term entries (plist) with three tile ids each (plist_t).
        // Distributed factorisation: list A (launch 0) holds this rank's subtree columns and its contributions to
        // the top, list B (launch 1) the top columns (updated from top panels only: the subtrees' updates are summed
        // into the top tiles between the launches) and the back substitution of the top and this rank's columns.
#ifndef LBA_CF_LA_MAX_LIST   // (A/B builds only, scripts/exp_build.sh)
#define LBA_CF_LA_MAX_LIST 16
#endif
        {
            struct TaskList {
                std::vector<int> tasks, task_i, task_t, pl0{0}, plist, plist_t;
            } LA, LB;
            TaskList* cur = &LA;
            std::vector<int>&tasks = LA.tasks, &task_i = LA.task_i, &task_t = LA.task_t, &pl0 = LA.pl0, &plist = LA.plist,
                            &plist_t = LA.plist_t;
            auto add_task = [&](int j, int i, int kind, int la, int t0, int t1, int t2, int t3, int t4) {
                cur->tasks.push_back(j | (kind << 24) | (la << 28));
                cur->task_i.push_back(i);
                cur->task_t.push_back(t0); cur->task_t.push_back(t1); cur->task_t.push_back(t2); cur->task_t.push_back(t3);
                cur->task_t.push_back(t4);
            };
            auto add_entry = [&](int e, int t0, int t1, int t2) {
                cur->plist.push_back(e);
                cur->plist_t.push_back(t0); cur->plist_t.push_back(t1); cur->plist_t.push_back(t2);
            };
            auto end_task = [&]() { cur->pl0.push_back((int)cur->plist.size()); };
            // (split) the panels whose updates a column of owner o takes inside its launch: its own subtree's, or the
            // top's for a top column
            auto same_part = [&](int pp, int o) { return !split || own[pp] == o; };
            const std::vector<int>& rank = pl.rank;
            auto by_rank = [&](int x, int y) { return rank[x] < rank[y]; };
            // row c's columns below the diagonal
            auto rowcols = [&](int c) {
                return std::vector<int>(pl.cols.begin() + pl.rowptr[c], pl.cols.begin() + pl.rowptr[c + 1] - 1);
            };
            // structure of L^-1 (L^-1 solve only): Linv(i,j) != 0 iff some k in [j, i) with L(i,k) != 0 has
            // Linv(k,j) != 0
            std::vector<std::vector<char>> nzi(band ? 0 : NP, std::vector<char>(band ? 0 : NP, 0));
            for (int i = 0; !band && i < NP; ++i) {
                nzi[i][i] = 1;
                const std::vector<int> rc = rowcols(i);
                for (int j = 0; j < i; ++j)
                    for (int k : rc)
                        if (k >= j && nzi[k][j]) { nzi[i][j] = 1; break; }
            }
            // band mode visits the columns in update order (the halves of every dissection level side by
            // side), so they are factored and substituted concurrently
            for (int cq = 0; cq < NP; ++cq) {
                const int c = band ? pl.uord[cq] : cq;
                if (split && own[c] >= 0 && own[c] != p->part_rank) continue;   // another rank's subtree
                cur = (split && own[c] < 0) ? &LB : &LA;
                std::vector<int> rcc;
                for (int pp : rowcols(c))
                    if (same_part(pp, own[c])) rcc.push_back(pp);
                std::vector<int> rows(1, c);
                rows.insert(rows.end(), pl.colrows[c].begin(), pl.colrows[c].end());
                for (int i : rows) {   // factor tiles of column c (the diagonal first)
                    // lookahead over k = c - 1 when tile (c, k) exists and k is the last update of A(c, c)
                    // in update order (then every copy of a tile sees the same update order)
                    // and only in dense mode, on a short list of its own: a lookahead task applies 5 tile products
                    // per entry instead of 2.  A band-mode solve has thousands of tasks on 512 workgroups, so the
                    // redundant products of column k cost more than the hand-off they save (config 2's solve
                    // 465 -> 357 us, config 4's 3.25 -> 2.25 ms without them, profiles/r8p_ab_lookahead.txt);
                    // config 1's few tasks (dense mode, lists <= 16) keep it: it is their chain.  (The band
                    // kernel, k_chol_flow_band, has no lookahead path.)
                    const int k = c - 1;
                    bool la = k >= 0 && pl.nz(c, k) && same_part(k, own[c]) && !band &&
                              (int)rcc.size() <= LBA_CF_LA_MAX_LIST;
                    for (int pp : rcc)
                        if (la && pp != k && rank[pp] > rank[k]) la = false;
                    const int tcc = pl.tile_id(c, c), tic = i == c ? -1 : pl.tile_id(i, c);
                    if (la) {
                        const int tik = pl.tile_id(i, k);
                        add_task(c, i, 0, 1, tcc, tic, pl.tile_id(k, k), pl.tile_id(c, k), i == c ? -1 : tik);
                        // updates of the held tiles A(c,c), A(i,c), A(k,k), A(c,k), A(i,k) from panels p < k
                        std::vector<int> ps;
                        for (int pp : rcc) if (pp < k) ps.push_back(pp);
                        for (int pp : rowcols(k))
                            if (same_part(pp, own[c])) ps.push_back(pp);
                        std::sort(ps.begin(), ps.end());
                        ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
                        std::sort(ps.begin(), ps.end(), by_rank);
                        // column k is factored as soon as its own updates are in: bit 27 marks the last entry that
                        // updates row k (entries after it update rows c / i only, e.g. the other half's panels in a
                        // separator's first column); no such entry: before the first one (task bit 29)
                        int klast = -1;
                        for (int pp : ps) {   // only panels that update a held tile; row i only where used
                            const int tcp = pl.tile_id(c, pp), tkp = pl.tile_id(k, pp), tip = pl.tile_id(i, pp);
                            const bool fj = tcp >= 0, fk = tkp >= 0, fi = i != c && tip >= 0 && (fj || fk);
                            if (fk) klast = (int)cur->plist.size();
                            if (fj || fk) add_entry(pp | (fi << 24) | (fj << 25) | (fk << 26), tcp, fi ? tip : -1, tkp);
                        }
                        if (klast >= 0) cur->plist[klast] |= 1 << 27;
                        else cur->tasks.back() |= 1 << 29;
                    } else {
                        add_task(c, i, 0, 0, tcc, tic, -1, -1, -1);
                        std::vector<int> ps(rcc);
                        std::sort(ps.begin(), ps.end(), by_rank);
                        for (int pp : ps) {
                            const int tip = i == c ? -1 : pl.tile_id(i, pp);
                            add_entry(pp | ((tip >= 0) << 24), pl.tile_id(c, pp), tip, -1);
                        }
                    }
                    end_task();
                }
                if (band) {   // forward substitution y_c = L_cc^-1 (b_c - sum_k L(c,k) y_k), k in update order
                    add_task(c, c, 4, 0, pl.tile_id(c, c), -1, -1, -1, -1);
                    std::vector<int> ks(rcc);
                    std::sort(ks.begin(), ks.end(), by_rank);
                    for (int kk : ks) add_entry(kk, pl.tile_id(c, kk), -1, -1);
                    end_task();
                    continue;
                }
                for (int j = 0; j < c; ++j) {    // L^-1 tiles of row c: terms k ascending
                    if (!nzi[c][j]) continue;
                    add_task(j, c, 1, 0, -1, -1, -1, -1, -1);
                    for (int kk : rcc)
                        if (kk >= j && nzi[kk][j]) add_entry(kk, pl.tile_id(c, kk), -1, -1);
                    end_task();
                }
                if (c == NP - 1) {
                    // the last panel: y_c = L_cc^-1 (b_c - sum_k L(c,k) y_k) as a substitution task (kind 4): every
                    // y_k is out well before L_cc is, so y_c follows L_cc^-T at once instead of waiting for the
                    // L^-1 tiles of the last row and their shares
                    add_task(c, c, 4, 0, pl.tile_id(c, c), -1, -1, -1, -1);
                    std::vector<int> ks(rcc);
                    std::sort(ks.begin(), ks.end(), by_rank);
                    for (int kk : ks) add_entry(kk, pl.tile_id(c, kk), -1, -1);
                    end_task();
                    continue;
                }
                add_task(c, c, 3, 0, -1, -1, -1, -1, -1);   // y_c: the nonzero tiles of row c of L^-1
                for (int kk = 0; kk <= c; ++kk)
                    if (nzi[c][kk]) add_entry(kk, -1, -1, -1);
                end_task();
            }
            if (split) {
                // this rank's contributions to the top: per top tile (i, j) the sum over its subtree panels p of
                // L(i,p) L(j,p)^T, per top panel i the sum of L(i,p) y_p (kinds 6, 7)
                cur = &LA;
                for (int j = 0; j < NP; ++j) {
                    if (own[j] >= 0) continue;
                    std::vector<int> rows(1, j);
                    rows.insert(rows.end(), pl.colrows[j].begin(), pl.colrows[j].end());
                    for (int i : rows) {
                        std::vector<int> ps;
                        for (int pp : rowcols(j))
                            if (own[pp] == p->part_rank && pl.nz(i, pp)) ps.push_back(pp);
                        if (ps.empty()) continue;
                        std::sort(ps.begin(), ps.end(), by_rank);
                        add_task(j, i, 6, 0, pl.tile_id(i, j), -1, -1, -1, -1);
                        for (int pp : ps) add_entry(pp, pl.tile_id(j, pp), pl.tile_id(i, pp), -1);
                        end_task();
                    }
                    std::vector<int> ks;
                    for (int pp : rowcols(j))
                        if (own[pp] == p->part_rank) ks.push_back(pp);
                    if (ks.empty()) continue;
                    std::sort(ks.begin(), ks.end(), by_rank);
                    add_task(j, j, 7, 0, -1, -1, -1, -1, -1);
                    for (int pp : ks) add_entry(pp, pl.tile_id(j, pp), -1, -1);
                    end_task();
                }
                cur = &LB;
            }
            if (band) {
                // back substitution x_j = L_jj^-T (y_j - sum_i L(i,j)^T x_i) over the rows i > j of column j,
                // columns in reverse update order, terms in the order their x_i complete
                for (int cq = NP - 1; cq >= 0; --cq) {
                    const int j = pl.uord[cq];
                    if (split && own[j] >= 0 && own[j] != p->part_rank) continue;
                    add_task(j, j, 5, 0, -1, -1, -1, -1, -1);
                    std::vector<int> is(pl.colrows[j]);
                    std::sort(is.begin(), is.end(), [&](int x, int y) { return rank[x] > rank[y]; });
                    for (int i : is) add_entry(i, pl.tile_id(i, j), -1, -1);
                    end_task();
                }
            }
            for (int j = 0; !band && j < NP; ++j) {      // solution blocks: rows i >= j of column j of L^-1
                add_task(j, j, 2, 0, -1, -1, -1, -1, -1);
                for (int i = j; i < NP; ++i)
                    if (nzi[i][j]) add_entry(i, -1, -1, -1);
                end_task();
            }
            if (NP >= (1 << 24)) throw ApiError{LBA_E_LIMIT, "internal: too many panels for the dataflow factorisation"};
            D.cf_tasks = dupload(p, tasks);
            D.cf_task_i = dupload(p, task_i);
            D.cf_task_t = dupload(p, task_t);
            D.cf_ntasks = (int)tasks.size();
            D.cf_split = split ? 1 : 0;
            D.cf_ntasks2 = 0;
            if (split) {
                D.cf_tasks2 = dupload(p, LB.tasks);
                D.cf_task_i2 = dupload(p, LB.task_i);
                D.cf_task_t2 = dupload(p, LB.task_t);
                D.cf_pl02 = dupload(p, LB.pl0);
                D.cf_plist2 = dupload(p, LB.plist);
                D.cf_plist_t2 = dupload(p, LB.plist_t);
                D.cf_ntasks2 = (int)LB.tasks.size();
                p->split_tasks[0] = D.cf_ntasks;
                p->split_tasks[1] = D.cf_ntasks2;
            }
            // band mode: no L^-1 tiles (ivready unused: x_j goes to the back tasks as granules, cf_xg)
            const size_t niv = band ? (size_t)NP + 1 : (size_t)std::max(NP * (NP + 1) / 2, 1);
            D.cf_linv = band ? nullptr : dalloc<double>(p, (size_t)npad * npad);
            D.cf_ivready = dalloc<int>(p, niv);
            zero_later(p, D.cf_ivready, sizeof(int) * niv);
            D.cf_xg = band ? dalloc<unsigned long long>(p, 2 * (size_t)npad) : nullptr;
            if (band) zero_later(p, D.cf_xg, sizeof(unsigned long long) * 2 * (size_t)npad);
            D.cf_pl0 = dupload(p, pl0);
            D.cf_plist = dupload(p, plist);
            D.cf_plist_t = dupload(p, plist_t);
            D.cf_lready = dalloc<int>(p, std::max(ntile, 1));
            D.cf_dready = dalloc<int>(p, std::max(NP, 1));
            D.cf_fready = dalloc<int>(p, std::max(NP, 1));
            zero_later(p, D.cf_fready, sizeof(int) * std::max(NP, 1));
            D.cf_zready = dalloc<int>(p, std::max(NP, 1));
            zero_later(p, D.cf_zready, sizeof(int) * std::max(NP, 1));
            D.cf_zv = band ? nullptr : dalloc<double>(p, std::max((size_t)NP * NP * CHOL_NB, (size_t)1));
            D.cf_head = dalloc<unsigned long long>(p, 2);   // (ticket counters of the split's two launches)
            D.cf_abort = dalloc<int>(p, 1);
            zero_later(p, D.cf_lready, sizeof(int) * std::max(ntile, 1));
            zero_later(p, D.cf_dready, sizeof(int) * std::max(NP, 1));
            zero_later(p, D.cf_head, 2 * sizeof(unsigned long long));
            zero_later(p, D.cf_abort, sizeof(int));
        }
        sub("  flow tasks");
        D.cf_rowptr = dupload(p, pl.rowptr);
        D.cf_cols = dupload(p, pl.cols);
        D.ppos = dupload(p, ppos);
        D.pnat = dupload(p, pnat);
        D.rpos = dupload(p, rpos);
        D.rnat = dupload(p, rnat);
        // every trial, k_lin_schur zeroes S (the tiles of L: structural non-zeros and fill-in) and k_assemble
        // then writes the structurally non-zero blocks
        // (in decreasing order of the slots a block sums: the blocks outnumber k_assemble's resident workgroups
        // and the diagonal blocks sum the most partials, so they go first, as k_lin_schur's tiles do)
        std::vector<int> asm_list;
        for (int u = 0; u < n_ublocks; ++u)
            if (hcnt[u] > 0 || scnt[u] > 0 || ub_i[u] == ub_j[u]) asm_list.push_back(u);
        if (!std::getenv("LBA_DISPATCH_INDEX_ORDER"))
            std::stable_sort(asm_list.begin(), asm_list.end(),
                             [&](int x, int y) { return hcnt[x] + scnt[x] > hcnt[y] + scnt[y]; });
        D.n_ztiles = ntile;
        D.part_rank = p->part_rank;
        D.part_n = p->part_n;
        {   // natural row -> the rank that adds its once-per-system terms (-1: rank 0)
            std::vector<int> row_own(npad);
            for (int r = 0; r < npad; ++r) row_own[r] = own[ppos[r / CHOL_NB]];
            D.row_own = dupload(p, row_own);
        }
        std::vector<int> top_tiles;   // (split) the tiles of L in the top columns
        if (split)
            for (int i = 0; i < NP; ++i)
                for (int q = pl.rowptr[i]; q < pl.rowptr[i + 1]; ++q)
                    if (own[pl.cols[q]] < 0) top_tiles.push_back(q);
        D.n_top_tiles = (int)top_tiles.size();
        D.top_tiles = split ? dupload(p, top_tiles) : nullptr;
        if (p->part_n > 0) {
            // bS, b_p (replicated solve: S is all-reduced in place; split: the top tiles lead the buffer)
            D.n_env = (long long)D.n_top_tiles * CHOL_NB * CHOL_NB + npad + p->np;
            D.env_buf = dalloc<double>(p, (size_t)D.n_env);
            D.red4 = dalloc<double>(p, RED_N);
        }
        D.asm_list = dupload(p, asm_list);
        D.n_asm = (int)asm_list.size();
    }
    D.npad = npad;
    // S and L: packed envelope tiles (memory O(envelope); the natural-order dense H_pp of lba_linearize
    // goes to Sfull, allocated on first use)
    const size_t n_env_doubles = (size_t)D.n_ztiles * CHOL_NB * CHOL_NB;
    p->s_bytes = 2 * n_env_doubles * sizeof(double);
    sub("  envelope + assembly lists");
    D.Lm = dalloc<double>(p, n_env_doubles + 1);
    D.LinvT = dalloc<double>(p, (size_t)npad * CHOL_NB + 1);
    // Hpl: only the heavy landmarks' canonical pairs, then the segment pairs (regular tiles keep theirs in LDS)
    D.hpl_base = lm_pair0[n_reg];
    D.n_hpl = n_pairs - D.hpl_base + n_segpairs;
    D.Hpl = dalloc<double>(p, (size_t)36 * std::max(D.n_hpl, 1));
    D.Hll = dalloc<double>(p, (size_t)9 * std::max(nl + n_seg, 1));               // landmarks, then segments
    D.n_lm_all = nl + n_seg;
    D.bl = dalloc<double>(p, (size_t)3 * std::max(nl + n_seg, 1));
    D.Dinv = dalloc<double>(p, (size_t)9 * std::max(nl, 1));
    D.S = dalloc<double>(p, n_env_doubles + 1);
    D.Sfull = nullptr;
    D.Sdiag = dalloc<double>(p, (size_t)p->np + 1);
    D.bp = dalloc<double>(p, p->np + 1);
    D.xsol = dalloc<double>(p, npad + 1);
    D.bS = dalloc<double>(p, npad + 1);
    zero_later(p, D.bS, sizeof(double) * (npad + 1));
    D.yv = dalloc<double>(p, npad + 1);
    // S and L start zero (k_assemble writes the identity of the padding rows every time)
    zero_later(p, D.S, sizeof(double) * (n_env_doubles + 1));
    zero_later(p, D.Lm, sizeof(double) * (n_env_doubles + 1));
    zero_later(p, D.xsol, sizeof(double) * (npad + 1));
    D.x = dalloc<double>(p, p->np + 3 * (size_t)nl + 1);
    zero_later(p, D.x, sizeof(double) * (p->np + 3 * (size_t)nl + 1));   // BlockSolver::_x before any solve
    const int nchi = n_tiles + D.n_prior + D.n_vel + D.n_eprior;
    D.chi_lin = dalloc<double>(p, nchi + 1);
    D.n_chi = nchi;
    D.chi_eval = dalloc<double>(p, nchi + 1);
    // k_update: one workgroup per GP pair, KFs at 64 per workgroup, one per regular tile, heavy landmarks at 64
    D.n_upd_blocks = D.n_gp + (n_kfs + 63) / 64 + n_stiles + (n_heavy + 63) / 64;
    if (D.n_upd_blocks == 0) D.n_upd_blocks = 1;
    D.scale_part = dalloc<double>(p, D.n_upd_blocks);
    // the trial evaluation fused into k_update (LBA_NO_FUSED_EVAL: k_eval after it): not with heavy landmarks (their
    // segment tiles and trial states are other workgroups') nor free extrinsics (the trial camera records); only
    // when the whole k_update grid is resident at once (its evaluating workgroups wait for its producers), and
    // not for partitioned problems (ranks of an in-process group share one device)
    D.f32res = (p->cfg.flags & LBA_FLAG_F32_RESIDUAL) ? 1 : 0;
    D.fuse_eval = (n_heavy == 0 && n_ext == 0 && p->part_n == 0 && std::getenv("LBA_NO_FUSED_EVAL") == nullptr) ? 1 : 0;
    if (D.fuse_eval) {
        // (the occupancy of k_update on this device, computed once per device ordinal; the guarantee is for one
        // k_update launch on the device at a time -- problems of an in-process group, which share a device, never
        // fuse -- see include/amc_lba.h, lba_set_problem)
        static std::mutex res_mu;
        static std::map<int, int> resident_of;
        int resident;
        {
            std::lock_guard<std::mutex> lk(res_mu);
            auto it = resident_of.find(p->cfg.device);
            if (it == resident_of.end()) it = resident_of.emplace(p->cfg.device, update_resident_blocks(p->cfg.device)).first;
            resident = it->second;
        }
        if (update_grid(D, 1) > resident) D.fuse_eval = 0;
    }
    {   // the producer of every pose sample (fused evaluation): its GP pair, or the KF block of a KF pose sample
        const int nkb = (n_kfs + UPD_BLOCK_KFS - 1) / UPD_BLOCK_KFS;
        std::vector<int> prod(std::max(D.n_smp, 1), -1);
        for (int g = 0; g < D.n_gp; ++g)
            for (int s = gp_s0[g]; s < gp_s0[g + 1]; ++s) prod[s] = g;
        for (int k = 0; k < n_kfs; ++k) prod[D.n_gps + k] = D.n_gp + k / UPD_BLOCK_KFS;
        D.smp_prod = dupload(p, prod);
        D.upd_flag = dalloc<int>(p, (size_t)FLAG_STRIDE * (D.n_gp + nkb + 1));
        zero_later(p, D.upd_flag, sizeof(int) * FLAG_STRIDE * (D.n_gp + nkb + 1));
        p->upd_epoch = 0;
    }
    // k_expand + k_assemble of a trial in one launch (LBA_NO_FUSED_ASM: two): not with heavy landmarks (their merge
    // is k_expand's), partitioned problems or the fused factorisation flow (which assembles S itself)
    D.fuse_asm = (n_heavy == 0 && p->part_n == 0 && std::getenv("LBA_NO_FUSED_ASM") == nullptr) ? 1 : 0;
    D.hs_prod = dupload(p, hs_prod);
    D.gs_prod = dupload(p, gs_prod);
    D.exp_flag = dalloc<int>(p, (size_t)FLAG_STRIDE * std::max(D.n_smp, 1));
    zero_later(p, D.exp_flag, sizeof(int) * FLAG_STRIDE * std::max(D.n_smp, 1));
    p->asm_epoch = 0;
    D.info = dalloc<int>(p, 1);
    D.fault = dalloc<int>(p, 1);
    zero_later(p, D.fault, sizeof(int));
    D.ctl = dalloc<LMCtl>(p, 1);
    D.fin = dalloc<double>(p, 4);
    D.ob_chi2 = dalloc<double>(p, std::max(n_obs, 1));
    D.ob_res = dalloc<double>(p, 3 * (size_t)std::max(n_obs, 1));
    D.depth_ok = dalloc<unsigned char>(p, std::max(n_obs, 1));
    zero_later(p, D.info, sizeof(int));
    for (int s = 0; s < 2; ++s) {
        p->kst[s] = dalloc<double>(p, kst.size());
        p->lst[s] = dalloc<double>(p, lst.size());
        upload_into(p, p->kst[s], kst);
        upload_into(p, p->lst[s], lst);
        D.kbuf[s] = p->kst[s];
        D.lbuf[s] = p->lst[s];
    }
    zero_later(p, D.ctl, sizeof(LMCtl));
    flush_zero_ranges(p);
    flush_uploads(p);
    HIPCHK(hipStreamSynchronize(p->stream));   // the staged uploads (dupload) have landed, the ranges are zero
    mark("solve layout");
    p->cur = 0;
    p->has_problem = true;
    p->gps_fresh[0] = p->gps_fresh[1] = false;
    p->linearized = false;
    return LBA_OK;
}

// ------------------------------------------------------------------------------------------------
// computeActiveErrors + buildSystem at the current state (no elimination): H_pp / b_p pieces, Hpl,
// Hll, bl (lba_linearize, computeLambdaInit)
// the set-up's zero ranges in one launch: the (address, words) list is staged like every other upload, then the
// kernel clears every range after the flush that carries the list
void flush_zero_ranges(lba_problem* p) {
    if (p->zero_list.empty()) return;
    const int n = (int)(p->zero_list.size() / 2);
    size_t words = 0;
    for (int k = 0; k < n; ++k) words += p->zero_list[2 * k + 1];
    const unsigned long long* d = dupload(p, p->zero_list);
    flush_uploads(p);
    launch_zero_ranges(d, n, words, p->stream);
    HIPCHK(hipGetLastError());
    p->zero_list.clear();
}

void linearize(lba_problem* p, int write_res) {
    const DevProblem& D = p->D;
    if (!p->gps_fresh[p->cur]) launch_gp_prep(D, p->cur, 1, GATE_NONE, p->stream);
    p->gps_fresh[p->cur] = true;
    launch_lin_schur(D, p->cur, GATE_NONE, 0.0, LS_EDGES | (write_res ? LS_RES : 0), p->stream);
    launch_expand(D, p->cur, GATE_NONE, 0.0, 0, p->stream);
    HIPCHK(hipGetLastError());
    p->linearized = true;
}

// A bounded in-launch wait gave up (DevProblem::fault, never expected): the data it waited for may be stale, so
// the call fails instead of returning results computed from it; the word is cleared for the next call
[[noreturn]] void throw_fault(lba_problem* p, int code) {
    HIPCHK(hipStreamSynchronize(p->stream));
    // (on the problem's own stream, which is non-blocking: a null-stream memset would not be ordered before the next
    // call's kernels)
    HIPCHK(hipMemsetAsync(p->D.fault, 0, sizeof(int), p->stream));
    HIPCHK(hipStreamSynchronize(p->stream));
    throw ApiError{LBA_E_TIMEOUT, std::string("a device hand-off wait timed out (") +
                                      ((code & FAULT_FLOW) ? " factorisation" : "") + ((code & FAULT_EXP) ? " assembly" : "") +
                                      ((code & FAULT_UPD) ? " trial evaluation" : "") +
                                      " ); the problem's state is undefined until the next lba_set_problem"};
}
// the same check after calls that do not publish a trial summary (one 4-byte read after the stream's work)
void check_fault(lba_problem* p) {
    int f = 0;
    HIPCHK(hipMemcpyAsync(&f, p->D.fault, sizeof(int), hipMemcpyDeviceToHost, p->stream));
    HIPCHK(hipStreamSynchronize(p->stream));
    if (f) throw_fault(p, f);
}

// poll the published sequence number (see finalize_and_wait)
void wait_seq(lba_problem* p, unsigned long long seq) {
    volatile unsigned long long* flag = reinterpret_cast<volatile unsigned long long*>(p->h_fin + 4);
    for (unsigned it = 1; *flag != seq; ++it) {
        if ((it & 1023) == 0) {
            const hipError_t e = hipStreamQuery(p->stream);
            if (e != hipSuccess && e != hipErrorNotReady) throw HipError{e, "trial kernels"};
            if (e == hipSuccess && *flag != seq) throw HipError{hipErrorUnknown, "trial summary not published"};
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (p->h_fin[5] != 0.0) throw_fault(p, (int)p->h_fin[5]);
}

// Publish the trial summary (k_finalize writes it into host-mapped memory) and wait for it by
// polling its sequence number; the stream is queried now and then so a device fault is reported
// instead of spinning forever.  sync: also synchronise the stream (callers that copy device
// buffers afterwards, or read timing events).
// eval_sel >= 0: evaluate that state buffer first (k_eval).
void launch_fin(lba_problem* p, unsigned long long seq, int mode);

void finalize_and_wait(lba_problem* p, bool sync, int eval_sel = -1) {
    const unsigned long long seq = ++p->fin_seq;
    if (eval_sel >= 0) launch_eval(p->D, eval_sel, GATE_NONE, seq, FIN_NONE, p->stream);
    launch_fin(p, seq, FIN_HOST);
    HIPCHK(hipGetLastError());
    wait_seq(p, seq);
    if (sync) HIPCHK(hipStreamSynchronize(p->stream));
}


// k_assemble into S (ASM_SCHUR: the factorisation-order packed envelope a trial factors), Sfull (ASM_FULL:
// the natural dense H_pp of lba_linearize) or Sdiag (ASM_DIAG: its diagonal, computeLambdaInit)
void assemble_layout(lba_problem* p, double lambda, int flags, int gate = GATE_NONE) {
    if (flags & ASM_FULL) {   // the dense natural-order H_pp (lba_linearize): its own buffer, made on first use
        if (!p->D.Sfull) p->D.Sfull = dalloc<double>(p, (size_t)p->np * p->np + 1);
        HIPCHK(hipMemsetAsync(p->D.Sfull, 0, sizeof(double) * ((size_t)p->np * p->np), p->stream));
    }
    launch_assemble(p->D, lambda, flags, gate, p->stream);
    if ((flags & ASM_SCHUR) && p->part_n > 0 && !p->D.cf_split) {   // sum the ranks' reduced systems
        launch_env_pack(p->D, 0, gate, p->stream);
        preduce(p, p->D.S, (int64_t)p->D.n_ztiles * CHOL_NB * CHOL_NB);   // the packed envelope, in place
        preduce(p, p->D.env_buf, p->D.n_env);
        launch_env_pack(p->D, 1, gate, p->stream);
    }
}

// The reduced system's solve: one k_chol_flow launch, or (distributed factorisation) the rank's subtrees and
// its contributions to the top, the all-reduce of the top tiles with bS / b_p, then the top and the back
// substitution (both launches under one epoch: the second reads the first one's published tiles).  e0 / e1:
// events on the first / last dispatch.
void launch_solve(lba_problem* p, hipEvent_t e0, hipEvent_t e1, int sel, double lambda) {
    const DevProblem& D = p->D;
    const unsigned epoch = ++p->cf_epoch;
    if (!D.cf_split) {
        launch_cholesky_solve(D, GATE_NONE, epoch, p->stream, e0, e1);
        return;
    }
    launch_cholesky_part(D, 0, epoch, p->stream, e0, nullptr);
    launch_env_pack(D, 0, GATE_NONE, p->stream);
    preduce(p, D.env_buf, D.n_env);
    launch_env_pack(D, 1, GATE_NONE, p->stream);
    launch_cholesky_part(D, 1, epoch, p->stream, nullptr, e1);
}

// k_finalize, after summing the ranks' trial sums when partitioned
void launch_fin(lba_problem* p, unsigned long long seq, int mode) {
    if (p->part_n > 0) {
        launch_partials(p->D, p->stream);
        preduce(p, p->D.red4, RED_N);
    }
    launch_finalize(p->D, seq, mode, p->stream);
}

// One trial: the linearisation at the current state fused with the landmark elimination (k_lin_schur),
// the reduced camera system, its solve, the update into the trial buffers and (evaluate) the trial
// state's errors.  Every trial linearises: after a rejected trial the state is the same, and the
// deterministic reductions reproduce the previous linearisation bit for bit (g2o keeps it).
// evs: phase events [5] (LBA_FLAG_TIME_PHASES); sweep: the dispatch events of k_lin_schur (ev 6, 7)
// and k_chol_flow (ev 8, 9).
void trial(lba_problem* p, double lambda, bool evaluate, hipEvent_t* evs, bool sweep, bool sync = true) {
    const DevProblem& D = p->D;
    const int nx = 1 - p->cur;
    if (!p->gps_fresh[p->cur]) launch_gp_prep(D, p->cur, 1, GATE_NONE, p->stream);
    p->gps_fresh[p->cur] = true;
    if (evs) HIPCHK(hipEventRecord(evs[0], p->stream));
    launch_lin_schur(D, p->cur, GATE_NONE, lambda, LS_SCHUR | LS_EDGES, p->stream, sweep ? p->ev[6] : nullptr,
                     sweep ? p->ev[7] : nullptr);
    if (evs) HIPCHK(hipEventRecord(evs[1], p->stream));
    if (D.fuse_asm) {
        launch_exp_asm(D, p->cur, GATE_NONE, lambda, ++p->asm_epoch, p->stream);
    } else {
        launch_expand(D, p->cur, GATE_NONE, lambda, 1, p->stream);
        assemble_layout(p, lambda, ASM_SCHUR, GATE_NONE);
    }
    if (evs) HIPCHK(hipEventRecord(evs[2], p->stream));
    launch_solve(p, sweep ? p->ev[8] : nullptr, sweep ? p->ev[9] : nullptr, p->cur, lambda);
    if (evs) HIPCHK(hipEventRecord(evs[3], p->stream));
    // (+ the trial state's pose samples, and with D.fuse_eval its errors)
    launch_update(D, lambda, p->cur, GATE_NONE, 1, p->stream, evaluate ? 1 : 0, ++p->upd_epoch);
    p->gps_fresh[nx] = true;
    if (evaluate && !D.fuse_eval) launch_eval(D, nx, GATE_NONE, 0, FIN_NONE, p->stream);
    if (evs) HIPCHK(hipEventRecord(evs[4], p->stream));
    finalize_and_wait(p, sync || evs || sweep);
    p->linearized = false;
}

double eval_current(lba_problem* p) {
    const DevProblem& D = p->D;
    // the samples the linearisation then uses (kept when the last trial's k_update made them: the queued
    // loop then evaluates the same samples as this one)
    if (!p->gps_fresh[p->cur]) launch_gp_prep(D, p->cur, 1, GATE_NONE, p->stream);
    p->gps_fresh[p->cur] = true;
    finalize_and_wait(p, true, p->cur);
    return p->h_fin[1];
}

double lambda_init(lba_problem* p) {   // computeLambdaInit (levenberg.cpp:171-185)
    if (p->cfg.lambda_init > 0) return p->cfg.lambda_init;
    const DevProblem& D = p->D;
    assemble_layout(p, 0.0, ASM_DIAG);
    std::vector<double> Sd((size_t)p->np + 1), Hll(9 * (size_t)std::max(D.n_lm, 1));
    if (p->np)
        HIPCHK(hipMemcpyAsync(Sd.data(), D.Sdiag, p->np * sizeof(double), hipMemcpyDeviceToHost, p->stream));
    HIPCHK(hipMemcpyAsync(Hll.data(), D.Hll, 9 * (size_t)D.n_lm * sizeof(double), hipMemcpyDeviceToHost, p->stream));
    HIPCHK(hipStreamSynchronize(p->stream));
    double m = 0.0;
    for (int i = 0; i < p->np; ++i) m = std::max(m, std::fabs(Sd[i]));
    for (int l = 0; l < D.n_lm; ++l)
        for (int d = 0; d < 3; ++d) m = std::max(m, std::fabs(Hll[9 * (size_t)l + 4 * d]));
    return p->cfg.tau * m;
}

float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.f;
    return ms;
}

// Queued optimisation: the same iterations as the host-driven loop in optimize() below, but the LM
// decisions are taken on the device (k_finalize / lm_decide on the LMCtl record), so the host enqueues
// one trial per remaining iteration without waiting for any outcome, and synchronises once per batch.
// Launches of a queued trial take their state buffer and damping from the controller; every trial
// relinearises inside k_lin_schur (see trial()), and the state-touching kernels of a trial are no-ops
// once the controller is done (the assembly and solve of such a trial only touch scratch buffers).  A batch is one trial per iteration still to run, which is exact
// when every trial is accepted; after rejected trials the next batch covers the rest (a trial
// completes at most one iteration and an iteration takes at most max_trials trials, so this
// terminates).  The starting-state evaluation and computeLambdaInit run in the queue too.
int optimize_queued(lba_problem* p, int iters, lba_stats* st) {
    lba_stats s{};
    const auto t0 = std::chrono::steady_clock::now();
    const DevProblem& D = p->D;
    const bool tsweep = (p->cfg.flags & LBA_FLAG_TIME_SWEEP) != 0;
    LMCtl c{};
    c.lambda = p->cfg.lambda_init > 0 ? p->cfg.lambda_init : 0.0;
    c.ni = 2.0;
    c.cur = p->cur;
    c.iters = iters;
    c.need_lin = 1;
    c.max_trials = p->cfg.max_trials;
    c.early_stop = p->cfg.early_stop;
    c.result = LBA_RESULT_OK;
    c.chi0_lin = 1;   // chi2 of the starting state: the first trial's, at its linearisation point (lm_decide)
    launch_ctl_init(D, c, p->stream);
    // starting state: poses + GP samples (with the Jacobian factors the first linearisation uses; a
    // previous queue left them for both state buffers)
    if (!p->gps_fresh[p->cur]) launch_gp_prep(D, p->cur, 1, GATE_NONE, p->stream);
    p->gps_fresh[p->cur] = true;
    int issued = 0;
    std::vector<char> timed(tsweep ? HLOG_CAP : 0, 0);   // trials whose dispatches carry events
    const LMCtl* hc = reinterpret_cast<const LMCtl*>(p->h_fin + 8);
    while (true) {
        const int n = iters - c.it;
        const int first = issued;
        const auto te0 = std::chrono::steady_clock::now();
        for (int k = 0; k < n; ++k, ++issued) {
            // LBA_FLAG_TIME_SWEEP: the dispatches of k_lin_schur and k_chol_flow carry events (their own
            // start / end timestamps); the trials that ran are read from the controller's log afterwards
            // (LBA_FLAG_TIME_SAMPLED: the 6th trial of every 10 of a batch, or its first in a short batch:
            // mid-batch trials, away from the start-up launches of an optimize call)
            const int samp = n >= 6 ? 5 : 0;
            const bool tq = tsweep && issued < HLOG_CAP &&
                            (!(p->cfg.flags & LBA_FLAG_TIME_SAMPLED) || (issued - first) % 10 == samp);
            if (tsweep && issued < HLOG_CAP) timed[issued] = tq;
            if (tq && p->qev.size() < 4 * (size_t)issued + 4) {
                const size_t old = p->qev.size();
                p->qev.resize(std::max<size_t>(4 * (size_t)issued + 4, 2 * old));
                for (size_t e = old; e < p->qev.size(); ++e) HIPCHK(hipEventCreate(&p->qev[e]));
            }
            hipEvent_t* qe = tq ? p->qev.data() + 4 * (size_t)issued : nullptr;
            if (issued == 0 && p->cfg.lambda_init <= 0) {   // computeLambdaInit reads H_pp / Hll of the start
                launch_lin_schur(D, SEL_CUR, GATE_TRIAL, 0.0, LS_EDGES, p->stream);
                launch_expand(D, SEL_CUR, GATE_TRIAL, 0.0, 0, p->stream);
                assemble_layout(p, 0.0, ASM_DIAG);
                launch_lambda_init(D, p->cfg.tau, p->stream);
            }
            launch_lin_schur(D, SEL_CUR, GATE_TRIAL, LAMBDA_CTL, LS_SCHUR | LS_EDGES, p->stream, qe ? qe[0] : nullptr,
                             qe ? qe[1] : nullptr);
            if (D.fuse_asm) {
                launch_exp_asm(D, SEL_CUR, GATE_TRIAL, LAMBDA_CTL, ++p->asm_epoch, p->stream);
            } else {
                launch_expand(D, SEL_CUR, GATE_TRIAL, LAMBDA_CTL, 1, p->stream);
                assemble_layout(p, LAMBDA_CTL, ASM_SCHUR, GATE_NONE);
            }
            launch_solve(p, qe ? qe[2] : nullptr, qe ? qe[3] : nullptr, SEL_CUR, LAMBDA_CTL);
            // the step, the trial state and its pose samples with their Jacobian factors: the next
            // trial's linearisation reads them (no preparation launch)
            launch_update(D, LAMBDA_CTL, SEL_CUR, GATE_TRIAL, 1, p->stream, 1, ++p->upd_epoch);
            if (!D.fuse_eval) launch_eval(D, SEL_NEXT, GATE_TRIAL, 0, FIN_NONE, p->stream);
            launch_fin(p, ++p->fin_seq, k == n - 1 ? FIN_QUEUED_PUBLISH : FIN_QUEUED);
            HIPCHK(hipGetLastError());
        }
        if (std::getenv("LBA_ENQ_TIMING"))
            std::fprintf(stderr, "enqueue %d trials: %.1f us/trial\n", n,
                         std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - te0).count() /
                             std::max(n, 1));
        wait_seq(p, p->fin_seq);
        std::memcpy(&c, hc, sizeof(LMCtl));
        if (tsweep) {
            HIPCHK(hipStreamSynchronize(p->stream));
            for (int q = first; q < issued && q < HLOG_CAP; ++q)
                if (p->h_log[q] && timed[q]) {
                    s.ms_k_linearize += elapsed(p->qev[4 * q], p->qev[4 * q + 1]);
                    s.n_k_linearize += 1;
                    s.ms_k_solve += elapsed(p->qev[4 * q + 2], p->qev[4 * q + 3]);
                    s.n_k_solve += 1;
                }
        }
        if (c.done || n <= 0) break;
    }
    HIPCHK(hipStreamSynchronize(p->stream));
    p->cur = c.cur;
    p->gps_fresh[0] = p->gps_fresh[1] = true;   // every state write of the queue came with its samples
    p->lambda = c.lambda;
    p->ni = c.ni;
    p->nBad = c.nbad;
    p->linearized = false;
    s.chi2_initial = c.chi0;
    s.iterations = c.it;
    s.trials = c.trials;
    s.solve_failures = c.failures;
    s.result = c.result;
    s.chi2_final = c.last_chi;
    s.lambda_final = c.lambda;
    s.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (st) *st = s;
    return c.it;
}

int optimize(lba_problem* p, int iters, volatile const int32_t* stop, lba_stats* st) {
    if (!p->has_problem) throw ApiError{LBA_E_ARG, "no problem set"};
    if (p->part_n > 0 && p->cfg.lambda_init <= 0)
        throw ApiError{LBA_E_ARG, "partitioned problems need lambda_init > 0 (computeLambdaInit is a max over ranks)"};
    lba_stats s{};
    if (p->np + 3 * p->n_lm_dev == 0) throw ApiError{LBA_E_EMPTY, "0 vertices to optimize"};
    if (!stop && iters > 0 && !(p->cfg.flags & (LBA_FLAG_TIME_PHASES | LBA_FLAG_HOST_LOOP)))
        return optimize_queued(p, iters, st);
    const auto t0 = std::chrono::steady_clock::now();
    // chi2 of the starting state: the first trial's at its linearisation point (as the queued loop takes it);
    // evaluated on its own only when no trial runs (a stop flag already set)
    bool have_chi0 = false;
    double last_chi = 0.0;
    int it = 0, result = LBA_RESULT_OK;
    const bool tphase = (p->cfg.flags & LBA_FLAG_TIME_PHASES) != 0;
    const bool tsweep = tphase || (p->cfg.flags & LBA_FLAG_TIME_SWEEP) != 0;
    for (int i = 0; i < iters; ++i) {
        if (stop && *stop) { result = LBA_RESULT_STOPPED; break; }
        if (i == 0) {
            if (p->cfg.lambda_init <= 0) linearize(p, 0);
            p->lambda = lambda_init(p);
            p->ni = 2.0;
            p->nBad = 0;
        }
        double currentChi = 0.0, iniChi = 0.0, rho = 0.0;
        int qmax = 0;
        do {
            trial(p, p->lambda, true, tphase ? p->ev : nullptr, tsweep, false);
            if (qmax == 0) currentChi = iniChi = p->h_fin[0];
            if (!have_chi0) { s.chi2_initial = p->h_fin[0]; have_chi0 = true; }
            if (tphase) {   // (ms_linearize: the fused linearisation + elimination)
                s.ms_linearize += elapsed(p->ev[0], p->ev[1]);
                s.ms_schur += elapsed(p->ev[1], p->ev[2]);
                s.ms_solve += elapsed(p->ev[2], p->ev[3]);
                s.ms_update_eval += elapsed(p->ev[3], p->ev[4]);
            }
            if (tsweep) {
                s.ms_k_linearize += elapsed(p->ev[6], p->ev[7]);
                s.n_k_linearize += 1;
                s.ms_k_solve += elapsed(p->ev[8], p->ev[9]);
                s.n_k_solve += 1;
            }
            double tempChi = p->h_fin[1];
            last_chi = tempChi;
            const bool ok2 = p->h_fin[3] == 0.0;
            if (!ok2) { tempChi = std::numeric_limits<double>::max(); s.solve_failures++; }
            rho = currentChi - tempChi;
            const double scale = p->h_fin[2] + 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                const double t3 = 2 * rho - 1;   // (2 rho - 1)^3 as in lm_decide (lba_kernels.hip)
                double alpha = 1. - t3 * t3 * t3;
                alpha = std::min(alpha, 2. / 3.);
                const double sf = std::max(1. / 3., alpha);
                p->lambda *= sf;
                p->ni = 2;
                currentChi = tempChi;
                p->cur = 1 - p->cur;   // discardTop: the trial state becomes current
            } else {
                p->lambda *= p->ni;
                p->ni *= 2;           // pop: keep the current state
            }
            qmax++;
        } while (rho < 0 && qmax < p->cfg.max_trials && !(stop && *stop));
        s.trials += qmax;
        ++it;
        result = LBA_RESULT_OK;
        if (qmax == p->cfg.max_trials || rho == 0) result = LBA_RESULT_TERMINATE;
        else if (p->cfg.early_stop) {
            if ((iniChi - currentChi) * 1e3 < iniChi) p->nBad++;
            else p->nBad = 0;
            if (p->nBad >= 3) result = LBA_RESULT_TERMINATE;
        }
        p->linearized = false;
        if (result != LBA_RESULT_OK && p->cfg.early_stop) break;
    }
    HIPCHK(hipStreamSynchronize(p->stream));
    if (!have_chi0) last_chi = s.chi2_initial = eval_current(p);
    s.iterations = it;
    s.result = result;
    s.chi2_final = last_chi;
    s.lambda_final = p->lambda;
    s.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (st) *st = s;
    return it;
}

int map_error(lba_problem* p, const HipError& e) {
    if (p) p->err = std::string(e.what) + ": " + hipGetErrorString(e.e);
    return LBA_E_HIP;
}

}  // namespace

// ==================================================================================================
// C ABI
struct GroupSlot {   // lba_set_partition_group: the user pointer of the in-process all-reduce
    lba_group* g;
    int rank;
};

static std::atomic<int> g_live_problems{0};   // lba_live_problems: engines created and not yet destroyed

extern "C" {

int lba_abi_version(void) { return LBA_ABI_VERSION; }

int lba_live_problems(void) { return g_live_problems.load(); }

int lba_debug_pool_stress(int32_t passes, int32_t max_pieces) {
    if (passes < 0 || max_pieces < 1) return LBA_E_ARG;
    int errors = 0;
    std::atomic<int> in_flight{0};
    std::vector<std::atomic<int>> runs((size_t)max_pieces);
    for (int pass = 0; pass < passes; ++pass) {
        // alternate short and long passes, so a pass with more pieces follows one with fewer
        const int n = 1 + (int)(((long long)pass * 7919 + (pass & 1) * (max_pieces / 2)) % max_pieces);
        for (int i = 0; i < n; ++i) runs[i].store(0, std::memory_order_relaxed);
        par_for(n, [&](int i) {
            in_flight.fetch_add(1, std::memory_order_acq_rel);
            runs[i].fetch_add(1, std::memory_order_acq_rel);
            for (int k = 0; k < (i * 37) % 97; ++k) __builtin_ia32_pause();
            in_flight.fetch_sub(1, std::memory_order_acq_rel);
        });
        if (in_flight.load(std::memory_order_acquire) != 0) ++errors;   // a piece outlived its pass
        for (int i = 0; i < n; ++i)
            if (runs[i].load(std::memory_order_acquire) != 1) ++errors;   // missed or run twice
    }
    return errors;
}

int lba_create(lba_problem** out, const lba_config* cfg) {
    if (!out || !cfg) return LBA_E_ARG;
    *out = nullptr;
    lba_problem* p = new lba_problem();
    p->cfg = *cfg;
    if (p->cfg.max_trials <= 0) p->cfg.max_trials = 10;
    if (p->cfg.tau <= 0) p->cfg.tau = 1e-5;
    try {
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        if (cfg->device < 0 || cfg->device >= ndev) {
            p->err = "invalid device";
            delete p;
            return LBA_E_ARG;
        }
        HIPCHK(hipSetDevice(cfg->device));
        HIPCHK(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
        for (auto& e : p->ev) HIPCHK(hipEventCreate(&e));
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&p->h_fin), HFIN_DOUBLES * sizeof(double),
                             hipHostMallocMapped | hipHostMallocCoherent));
        for (int i = 0; i < HFIN_DOUBLES; ++i) p->h_fin[i] = 0.0;
        HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&p->d_hfin), p->h_fin, 0));
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&p->h_log), HLOG_CAP * sizeof(int),
                             hipHostMallocMapped | hipHostMallocCoherent));
        for (int i = 0; i < HLOG_CAP; ++i) p->h_log[i] = 0;
        HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&p->d_hlog), p->h_log, 0));
    } catch (const HipError& e) {
        delete p;
        return LBA_E_HIP;
    }
    *out = p;
    g_live_problems.fetch_add(1);
    return LBA_OK;
}

void lba_destroy(lba_problem* p) {
    if (!p) return;
    g_live_problems.fetch_sub(1);
    (void)hipSetDevice(p->cfg.device);
    if (p->stream) (void)hipStreamSynchronize(p->stream);
    free_all(p);
    release_all(p);
    for (auto& e : p->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : p->qev)
        if (e) (void)hipEventDestroy(e);
    for (auto& a : p->pin_chunks) (void)hipHostFree(a.ptr);
    p->pin_chunks.clear();
    if (p->h_fin) (void)hipHostFree(p->h_fin);
    if (p->h_log) (void)hipHostFree(p->h_log);
    if (p->d_status) (void)hipFree(p->d_status);
    if (p->comm) (void)ncclCommDestroy(p->comm);
    if (p->farm_comm) (void)ncclCommDestroy(p->farm_comm);
    if (p->f_buf) (void)hipFree(p->f_buf);
    if (p->f_idx) (void)hipFree(p->f_idx);
    delete static_cast<GroupSlot*>(p->group_slot);
    delete static_cast<GroupSlot*>(p->farm_slot);
    if (p->stream) (void)hipStreamDestroy(p->stream);
    delete p;
}

int lba_set_config(lba_problem* p, const lba_config* cfg) {
    if (!p || !cfg) return LBA_E_ARG;
    if (cfg->device != p->cfg.device) {
        p->err = "lba_set_config cannot move a problem to another device";
        return LBA_E_ARG;
    }
    p->cfg = *cfg;
    if (p->cfg.max_trials <= 0) p->cfg.max_trials = 10;
    if (p->cfg.tau <= 0) p->cfg.tau = 1e-5;
    return LBA_OK;
}

const char* lba_last_error(const lba_problem* p) { return p ? p->err.c_str() : "null problem"; }

int lba_pose_dim(const lba_problem* p) { return p && p->has_problem ? p->np_ext : 0; }

int lba_debug_inject_fault(lba_problem* p, int32_t code) {
    if (!p || !p->has_problem || code <= 0 || code > (FAULT_FLOW | FAULT_EXP | FAULT_UPD)) return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        HIPCHK(hipMemcpyAsync(p->D.fault, &code, sizeof(int), hipMemcpyHostToDevice, p->stream));
        HIPCHK(hipStreamSynchronize(p->stream));
        return LBA_OK;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

int lba_get_cams(lba_problem* p, lba_cam* cams_out) {
    if (!p || !p->has_problem || !cams_out) return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        for (int c = 0; c < p->n_cam; ++c) cams_out[c] = p->cams[c];
        if (p->n_ext) {
            std::vector<double> kx(KF_STRIDE * (size_t)p->n_ext);
            HIPCHK(hipMemcpyAsync(kx.data(), p->kst[p->cur] + KF_STRIDE * (size_t)p->n_kf, kx.size() * sizeof(double),
                                  hipMemcpyDeviceToHost, p->stream));
            HIPCHK(hipStreamSynchronize(p->stream));
            for (int e = 0; e < p->n_ext; ++e) {
                lba_cam& o = cams_out[p->ext_cams[e]];
                for (int i = 0; i < 4; ++i) o.q[i] = kx[KF_STRIDE * e + i];
                for (int i = 0; i < 3; ++i) o.t[i] = kx[KF_STRIDE * e + 4 + i];
            }
        }
        return LBA_OK;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

int lba_set_partition(lba_problem* p, int32_t rank, int32_t nranks, lba_allreduce_fn fn, void* user) {
    if (!p || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !fn)) return LBA_E_ARG;
    if (p->has_problem) {
        p->err = "lba_set_partition must precede lba_set_problem";
        return LBA_E_ARG;
    }
    p->part_rank = rank;
    p->part_n = nranks > 1 ? nranks : 0;
    if (p->part_n > 0 && !p->d_status) {
        (void)hipSetDevice(p->cfg.device);
        if (hipMalloc(&p->d_status, sizeof(double)) != hipSuccess) {
            p->err = "hipMalloc of the partition status word failed";
            return LBA_E_HIP;
        }
    }
    p->red_fn = fn;
    p->red_user = user;
    return LBA_OK;
}

static int rccl_allreduce(double* buf, int64_t n, void* stream, void* user) {
    return ncclAllReduce(buf, buf, (size_t)n, ncclDouble, ncclSum, static_cast<ncclComm_t>(user),
                         static_cast<hipStream_t>(stream)) == ncclSuccess ? 0 : -1;
}

int lba_rccl_unique_id(void* id_out) {
    if (!id_out) return LBA_E_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return LBA_E_HIP;
    std::memcpy(id_out, &id, sizeof(id));
    return LBA_OK;
}

int lba_set_partition_rccl(lba_problem* p, const void* id, int32_t rank, int32_t nranks) {
    if (!p || !id) return LBA_E_ARG;
    if (nranks <= 1) return lba_set_partition(p, 0, 1, nullptr, nullptr);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    if (hipSetDevice(p->cfg.device) != hipSuccess) return LBA_E_HIP;
    ncclComm_t comm = nullptr;
    if (ncclCommInitRank(&comm, nranks, uid, rank) != ncclSuccess) {
        p->err = "ncclCommInitRank failed";
        return LBA_E_HIP;
    }
    const int rc = lba_set_partition(p, rank, nranks, rccl_allreduce, comm);
    if (rc != LBA_OK) {
        ncclCommDestroy(comm);
        return rc;
    }
    if (p->comm) ncclCommDestroy(p->comm);
    p->comm = comm;
    return LBA_OK;
}

// ---- in-process all-reduce across problems on one device (tests; lba_group)
constexpr int GROUP_MAX = 16;
struct GroupBufs {
    double* b[GROUP_MAX];
    int n;
};
__global__ void k_group_sum(GroupBufs g, long long count) {
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (long long)gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int r = 0; r < g.n; ++r) s += g.b[r][e];   // rank order: the same bits everywhere
        for (int r = 0; r < g.n; ++r) g.b[r][e] = s;
    }
}

}  // extern "C"

struct lba_group {
    int n = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    unsigned long long gen = 0;
    GroupBufs bufs{};
    long long count = -1;
    bool bad = false;
    hipStream_t rs = nullptr;
    hipEvent_t ev_in[GROUP_MAX] = {};
    hipEvent_t ev_done = nullptr;
};
static int group_allreduce(double* buf, int64_t n, void* stream, void* user) {
    GroupSlot* sl = static_cast<GroupSlot*>(user);
    lba_group* g = sl->g;
    hipStream_t st = static_cast<hipStream_t>(stream);
    std::unique_lock<std::mutex> lk(g->m);
    if (hipEventRecord(g->ev_in[sl->rank], st) != hipSuccess) g->bad = true;
    g->bufs.b[sl->rank] = buf;
    if (g->arrived == 0) g->count = n;
    else if (g->count != n) g->bad = true;
    const unsigned long long my = g->gen;
    if (++g->arrived == g->n) {   // last arrival: one sum kernel after every rank's stream point
        bool ok = !g->bad;
        for (int r = 0; r < g->n && ok; ++r) ok = hipStreamWaitEvent(g->rs, g->ev_in[r], 0) == hipSuccess;
        g->bufs.n = g->n;
        if (ok && n > 0) {
            const int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
            hipLaunchKernelGGL(k_group_sum, dim3(blocks), dim3(256), 0, g->rs, g->bufs, (long long)n);
            ok = hipGetLastError() == hipSuccess;
        }
        ok = ok && hipEventRecord(g->ev_done, g->rs) == hipSuccess;
        g->bad = !ok;
        g->arrived = 0;
        g->gen++;
        g->cv.notify_all();
    } else {
        // bounded: a peer that never arrives (it failed outside the set-up's status point) poisons the
        // group instead of hanging this rank
        if (!g->cv.wait_for(lk, std::chrono::seconds(120), [&] { return g->gen != my; })) {
            g->bad = true;
            return -1;
        }
    }
    const bool bad = g->bad;
    // every rank's stream waits for the sum (the event is re-recorded only after all ranks arrive again)
    if (bad || hipStreamWaitEvent(st, g->ev_done, 0) != hipSuccess) return -1;
    return 0;
}

extern "C" {

int lba_group_create(lba_group** out, int32_t nranks) {
    if (!out || nranks < 1 || nranks > GROUP_MAX) return LBA_E_ARG;
    lba_group* g = new lba_group();
    g->n = nranks;
    if (hipStreamCreateWithFlags(&g->rs, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_done, hipEventDisableTiming) != hipSuccess) {
        delete g;
        return LBA_E_HIP;
    }
    for (int r = 0; r < nranks; ++r)
        if (hipEventCreateWithFlags(&g->ev_in[r], hipEventDisableTiming) != hipSuccess) return LBA_E_HIP;
    *out = g;
    return LBA_OK;
}

void lba_group_destroy(lba_group* g) {
    if (!g) return;
    (void)hipStreamSynchronize(g->rs);
    for (int r = 0; r < g->n; ++r)
        if (g->ev_in[r]) (void)hipEventDestroy(g->ev_in[r]);
    if (g->ev_done) (void)hipEventDestroy(g->ev_done);
    if (g->rs) (void)hipStreamDestroy(g->rs);
    delete g;
}

int lba_set_partition_group(lba_problem* p, lba_group* g, int32_t rank) {
    if (!p || !g || rank < 0 || rank >= g->n) return LBA_E_ARG;
    GroupSlot* sl = new GroupSlot{g, rank};
    const int rc = lba_set_partition(p, rank, g->n, group_allreduce, sl);
    if (rc != LBA_OK) {
        delete sl;
        return rc;
    }
    delete static_cast<GroupSlot*>(p->group_slot);
    p->group_slot = sl;
    return LBA_OK;
}

// ---- window farm
int lba_setup_host_profile(const lba_config* cfg, const lba_kf* kfs, int32_t n_kf, const double* lm_xyz, int32_t n_lm,
                           const lba_obs* obs, int32_t n_obs, const lba_prior* priors, int32_t n_priors,
                           const int32_t* vel_kfs, int32_t n_vel, const lba_cam* cams, int32_t n_cam,
                           double phase_ms[3], int32_t counts[5]) {
    if (!cfg) return LBA_E_ARG;
    lba_problem p;   // no stream, no device memory: set_problem stops before its first device call
    p.cfg = *cfg;
    p.host_only = true;
    try {
        const int rc = set_problem(&p, kfs, n_kf, lm_xyz, n_lm, obs, n_obs, priors, n_priors, vel_kfs, n_vel, cams, n_cam);
        if (rc < 0) return rc;
    } catch (const ApiError& e) {
        return e.code;
    } catch (const HipError&) {
        return LBA_E_HIP;
    }
    for (int i = 0; i < 3; ++i) if (phase_ms) phase_ms[i] = i < (int)p.setup_ms.size() ? p.setup_ms[i] : 0.0;
    if (counts) {
        counts[0] = p.n_lm_dev;
        counts[1] = p.n_pb;
        counts[2] = p.np;
        counts[3] = p.setup_tiles;
        counts[4] = (int32_t)p.setup_hash;
    }
    return LBA_OK;
}

int lba_setup_phases(const lba_problem* p, double* ms, int32_t n) {
    if (!p || n < 0 || (n > 0 && !ms)) return LBA_E_ARG;
    const int32_t k = std::min<int32_t>(n, (int32_t)p->setup_ms.size());
    for (int32_t i = 0; i < k; ++i) ms[i] = p->setup_ms[i];
    return k;
}

int64_t lba_device_bytes(const lba_problem* p) {
    if (!p) return LBA_E_ARG;
    int64_t b = 0;
    for (size_t k = 0; k < p->alloc_cursor && k < p->allocs.size(); ++k) b += (int64_t)p->allocs[k].bytes;
    for (size_t k = 0; k < p->up_chunk && k < p->up_end.size(); ++k) b += (int64_t)p->up_end[k];   // (the window's
    b += (int64_t)p->up_off;                                                                          // read-only arrays)
    return b;
}

int lba_kernel_modes(const lba_problem* p, int32_t out[4]) {
    if (!p || !out || !p->has_problem) return LBA_E_ARG;
    out[0] = p->D.fuse_eval;
    out[1] = p->D.fuse_asm;
    out[2] = p->D.f32res;
    out[3] = update_grid(p->D, 1);
    return LBA_OK;
}

int lba_solver_info(const lba_problem* p, int32_t out[8]) {
    if (!p || !out || !p->has_problem) return LBA_E_ARG;
    out[0] = p->nd_tail;
    out[1] = p->D.npad / CHOL_NB;
    out[2] = p->D.n_ztiles;
    out[3] = p->D.cf_band;
    out[4] = p->chain;
    out[5] = p->nd_levels;
    out[6] = p->s_tiles;
    out[7] = p->D.n_ztiles - p->s_tiles;
    return LBA_OK;
}

int lba_partition_assign(const lba_config* cfg, const lba_kf* kfs, int32_t n_kf, int32_t n_lm, const lba_obs* obs,
                         int32_t n_obs, const lba_prior* priors, int32_t n_priors, const int32_t* vel_kfs, int32_t n_vel,
                         int32_t nranks, int32_t* lm_rank, int32_t* prior_rank, int32_t* vel_rank, int32_t* panels_out,
                         int32_t* kf_rank) {
    using namespace lba;
    if (!cfg || n_kf < 0 || n_lm < 0 || n_obs < 0 || n_priors < 0 || n_vel < 0 || nranks < 1 || (n_kf && !kfs) ||
        (n_obs && !obs) || (n_priors && !priors) || (n_vel && !vel_kfs) || (n_lm && !lm_rank) ||
        (n_priors && !prior_rank) || (n_vel && !vel_rank))
        return LBA_E_ARG;
    try {
        // pose blocks as a partitioned lba_set_problem numbers them: every non-fixed keyframe, in order
        std::vector<int> H(n_kf, -1);
        int n_pb = 0;
        for (int k = 0; k < n_kf; ++k)
            if (!kfs[k].fixed) H[k] = n_pb++;
        auto kf_ok = [&](int k) { return k >= 0 && k < n_kf; };
        for (int i = 0; i < n_obs; ++i)
            if (!kf_ok(obs[i].kf_b) || (is_gp(obs[i].kind) && !kf_ok(obs[i].kf_a)) || obs[i].lm < 0 || obs[i].lm >= n_lm)
                return LBA_E_ARG;
        for (int i = 0; i < n_priors; ++i)
            if (!kf_ok(priors[i].kf_a) || !kf_ok(priors[i].kf_b)) return LBA_E_ARG;
        for (int i = 0; i < n_vel; ++i)
            if (!kf_ok(vel_kfs[i])) return LBA_E_ARG;
        const int np = 12 * n_pb, NP = (np + CHOL_NB - 1) / CHOL_NB;
        // the pattern lba_set_problem plans: every pose block's diagonal, the blocks of every pair of a
        // landmark's keyframes, of every motion prior
        std::vector<std::vector<int>> blocks(n_lm);
        for (int i = 0; i < n_obs; ++i) {
            const lba_obs& o = obs[i];
            if (H[o.kf_b] >= 0) blocks[o.lm].push_back(H[o.kf_b]);
            if (is_gp(o.kind) && H[o.kf_a] >= 0) blocks[o.lm].push_back(H[o.kf_a]);
        }
        std::vector<std::vector<int>> lower(NP);
        for (int P = 0; P < NP; ++P) lower[P].push_back(P);
        auto couple_blocks = [&](int a, int b) {
            const int bi = std::min(a, b), bj = std::max(a, b);
            for (int dr : {0, 11})
                for (int dc : {0, 11}) {
                    const int r = 12 * bj + dr, c = 12 * bi + dc;
                    lower[std::max(r, c) / CHOL_NB].push_back(std::min(r, c) / CHOL_NB);
                }
        };
        for (auto& b : blocks) {
            std::sort(b.begin(), b.end());
            b.erase(std::unique(b.begin(), b.end()), b.end());
            for (size_t x = 0; x < b.size(); ++x)
                for (size_t y = x; y < b.size(); ++y) couple_blocks(b[x], b[y]);
        }
        for (int i = 0; i < n_priors; ++i) {
            const int a = H[priors[i].kf_a], b = H[priors[i].kf_b];
            if (a >= 0) couple_blocks(a, a);
            if (b >= 0) couple_blocks(b, b);
            if (a >= 0 && b >= 0) couple_blocks(a, b);
        }
        for (int i = 0; i < n_vel; ++i)
            if (H[vel_kfs[i]] >= 0) couple_blocks(H[vel_kfs[i]], H[vel_kfs[i]]);
        for (int P = 0; P < NP; ++P) {
            std::sort(lower[P].begin(), lower[P].end());
            lower[P].erase(std::unique(lower[P].begin(), lower[P].end()), lower[P].end());
        }
        const lba_plan::Plan pl = plan_panels(NP, NP, lower);
        const std::vector<int> own = lba_plan::split_subtrees(pl, nranks);
        // the rank of a set of pose blocks: the subtree its rows reach (one at most), else fallback
        auto rank_of = [&](std::initializer_list<int> hs, const std::vector<int>* more, int fallback) {
            int r = -1;
            auto visit = [&](int h) {
                if (h < 0) return;
                for (int row : {12 * h, 12 * h + 11}) {
                    const int o = own[pl.ppos[row / CHOL_NB]];
                    if (o >= 0) r = o;
                }
            };
            for (int h : hs) visit(h);
            if (more)
                for (int h : *more) visit(h);
            return r >= 0 ? r : fallback;
        };
        for (int l = 0; l < n_lm; ++l) lm_rank[l] = rank_of({}, &blocks[l], l % nranks);
        for (int i = 0; i < n_priors; ++i)
            prior_rank[i] = rank_of({H[priors[i].kf_a], H[priors[i].kf_b]}, nullptr, i % nranks);
        for (int i = 0; i < n_vel; ++i) vel_rank[i] = rank_of({H[vel_kfs[i]]}, nullptr, i % nranks);
        if (kf_rank)
            for (int k = 0; k < n_kf; ++k) kf_rank[k] = rank_of({H[k]}, nullptr, -1);
        if (panels_out) {
            std::vector<int> cnt(nranks, 0);
            int ntop = 0;
            for (int j = 0; j < NP; ++j) {
                if (own[j] < 0) ++ntop;
                else ++cnt[own[j]];
            }
            panels_out[0] = NP;
            panels_out[1] = ntop;
            panels_out[2] = *std::max_element(cnt.begin(), cnt.end());
        }
        return LBA_OK;
    } catch (const std::exception&) {
        return LBA_E_ARG;
    }
}

int lba_split_info(const lba_problem* p, double out[6]) {
    if (!p || !out || !p->has_problem) return LBA_E_ARG;
    const double tile = (double)CHOL_NB * CHOL_NB * sizeof(double);
    out[0] = p->flops_factor_rank;
    out[1] = p->flops_factor;
    // all-reduce bytes per trial: the split's (top tiles, bS, b_p) and the replicated solve's (every tile, bS, b_p)
    const double vec = (double)(p->D.npad + p->np) * sizeof(double);
    out[2] = p->part_n > 0 ? (p->D.cf_split ? p->D.n_top_tiles * tile + vec : p->D.n_ztiles * tile + vec) : 0.0;
    out[3] = p->D.n_ztiles * tile + vec;
    out[4] = p->split_panels[0];
    out[5] = p->split_panels[1];
    return LBA_OK;
}

int lba_kf_owner(const lba_problem* p, int32_t* owner) {
    if (!p || !owner || !p->has_problem) return LBA_E_ARG;
    const int n_kf = (int)p->kf_hidx.size() - p->n_ext;
    for (int k = 0; k < n_kf; ++k) {
        const int h = p->kf_hidx[k];
        int r = -1;
        if (h >= 0 && !p->split_own.empty())
            for (int row : {12 * h, 12 * h + 11}) {
                const int o = p->split_own[p->ppos_h[row / CHOL_NB]];
                if (o >= 0) r = o;
            }
        owner[k] = r;
    }
    return LBA_OK;
}

int lba_solver_flops(const lba_problem* p, double out[2]) {
    if (!p || !out || !p->has_problem) return LBA_E_ARG;
    out[0] = p->flops_factor;
    out[1] = 2.0 * 2.0 * (double)p->D.n_ztiles * CHOL_NB * CHOL_NB;   // forward + back substitution
    return LBA_OK;
}

int lba_set_farm(lba_problem* p, int32_t rank, int32_t nranks, lba_allreduce_fn fn, void* user) {
    if (!p || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !fn)) return LBA_E_ARG;
    if (p->farm_comm) (void)ncclCommDestroy(p->farm_comm);
    p->farm_comm = nullptr;
    delete static_cast<GroupSlot*>(p->farm_slot);
    p->farm_slot = nullptr;
    p->farm_rank = rank;
    p->farm_n = nranks;
    p->farm_fn = fn;
    p->farm_user = user;
    p->farm_planned = false;
    return LBA_OK;
}

int lba_set_farm_rccl(lba_problem* p, const void* id, int32_t rank, int32_t nranks) {
    if (!p || !id || nranks < 1 || rank < 0 || rank >= nranks) return LBA_E_ARG;
    if (nranks == 1) return lba_set_farm(p, 0, 1, nullptr, nullptr);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    if (hipSetDevice(p->cfg.device) != hipSuccess) return LBA_E_HIP;
    ncclComm_t comm = nullptr;
    if (ncclCommInitRank(&comm, nranks, uid, rank) != ncclSuccess) {
        p->err = "ncclCommInitRank failed (farm)";
        return LBA_E_HIP;
    }
    const int rc = lba_set_farm(p, rank, nranks, rccl_allreduce, comm);
    if (rc != LBA_OK) {
        ncclCommDestroy(comm);
        return rc;
    }
    p->farm_comm = comm;   // the exchange uses ncclAllGather on it directly
    return LBA_OK;
}

int lba_set_farm_group(lba_problem* p, lba_group* g, int32_t rank) {
    if (!p || !g || rank < 0 || rank >= g->n) return LBA_E_ARG;
    GroupSlot* sl = new GroupSlot{g, rank};
    const int rc = lba_set_farm(p, rank, g->n, group_allreduce, sl);
    if (rc != LBA_OK) {
        delete sl;
        return rc;
    }
    p->farm_slot = sl;
    return LBA_OK;
}

int lba_farm_match(int32_t rank, int32_t nranks, int32_t cap, const int64_t* pub_gid, const int64_t* gid,
                   const int32_t* owner, int32_t n, int32_t* src) {
    if (nranks < 1 || rank < 0 || rank >= nranks || cap < 0 || n < 0 || (n && (!gid || !owner || !src)) ||
        (cap && !pub_gid))
        return LBA_E_ARG;
    // one hash table per owner rank (its published ids -> position), built once per plan
    std::vector<std::unordered_map<int64_t, int>> pos(nranks);
    for (int r = 0; r < nranks; ++r) {
        if (r == rank) continue;
        for (int i = 0; i < cap; ++i) {
            const int64_t g = pub_gid[(size_t)r * cap + i];
            if (g >= 0) pos[r].emplace(g, i);
        }
    }
    int unmatched = 0;
    for (int i = 0; i < n; ++i) {
        src[i] = -1;
        const int o = owner[i];
        if (o < -1 || o >= nranks) return LBA_E_ARG;
        if (o < 0 || o == rank) continue;
        const auto it = pos[o].find(gid[i]);
        if (it == pos[o].end()) ++unmatched;
        else src[i] = o * cap + it->second;
    }
    return unmatched;
}

}  // extern "C"

namespace {
// all-gather of `stride` doubles per rank in place in buf (rank r's slot at buf + r stride) on the
// problem's stream: ncclAllGather, or the caller's sum all-reduce over slots that are zero but the own
void farm_gather(lba_problem* p, double* buf, int64_t stride) {
    if (p->farm_n <= 1) return;
    if (p->farm_comm) {
        if (ncclAllGather(buf + (size_t)p->farm_rank * stride, buf, (size_t)stride, ncclDouble, p->farm_comm,
                          p->stream) != ncclSuccess)
            throw ApiError{LBA_E_HIP, "farm all-gather (ncclAllGather) failed"};
    } else if (p->farm_fn(buf, stride * p->farm_n, (void*)p->stream, p->farm_user) != 0) {
        throw ApiError{LBA_E_HIP, "farm all-gather (all-reduce) failed"};
    }
}
template <typename T>
void farm_reserve(T** ptr, size_t* have, size_t bytes) {
    if (*have >= bytes) return;
    if (*ptr) HIPCHK(hipFree(*ptr));
    *ptr = nullptr;
    *have = 0;
    HIPCHK(hipMalloc(reinterpret_cast<void**>(ptr), bytes));
    *have = bytes;
}
}  // namespace

extern "C" {

int lba_farm_plan(lba_problem* p, const int64_t* kf_gid, const int32_t* kf_owner, const int64_t* lm_gid,
                  const int32_t* lm_owner, int32_t* out_counts) {
    if (!p || !p->has_problem || p->farm_n < 1 || (p->n_kf && (!kf_gid || !kf_owner)) ||
        (p->n_lm && (!lm_gid || !lm_owner)))
        return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        const int R = p->farm_n, me = p->farm_rank;
        std::vector<int> pub_kf, pub_lm;
        for (int k = 0; k < p->n_kf; ++k) {
            if (kf_owner[k] < -1 || kf_owner[k] >= R) throw ApiError{LBA_E_ARG, "farm plan: keyframe owner out of range"};
            if (kf_owner[k] == me) pub_kf.push_back(k);
        }
        for (int l = 0; l < p->n_lm; ++l) {
            if (lm_owner[l] < -1 || lm_owner[l] >= R) throw ApiError{LBA_E_ARG, "farm plan: landmark owner out of range"};
            if (lm_owner[l] == me && p->lm_dev[l] >= 0) pub_lm.push_back(l);   // (inactive: not on the device)
        }
        // 1. the ranks' published counts -> slot capacities
        double* tmp = nullptr;
        size_t tmp_bytes = 0;
        struct Tmp {
            double*& t;
            ~Tmp() { if (t) (void)hipFree(t); }
        } guard{tmp};
        std::vector<double> h(2 * (size_t)R, 0.0);
        h[2 * me] = (double)pub_kf.size();
        h[2 * me + 1] = (double)pub_lm.size();
        farm_reserve(&tmp, &tmp_bytes, h.size() * sizeof(double));
        HIPCHK(hipMemcpy(tmp, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
        farm_gather(p, tmp, 2);
        HIPCHK(hipStreamSynchronize(p->stream));
        HIPCHK(hipMemcpy(h.data(), tmp, h.size() * sizeof(double), hipMemcpyDeviceToHost));
        int kcap = 0, lcap = 0;
        for (int r = 0; r < R; ++r) {
            kcap = std::max(kcap, (int)h[2 * r]);
            lcap = std::max(lcap, (int)h[2 * r + 1]);
        }
        // 2. the published global ids (-1 padded), exchanged once; ids travel as doubles (exact below 2^53)
        const int gs = kcap + lcap;
        std::vector<double> g((size_t)R * gs, 0.0);
        for (int i = 0; i < kcap; ++i) g[(size_t)me * gs + i] = i < (int)pub_kf.size() ? (double)kf_gid[pub_kf[i]] : -1.0;
        for (int i = 0; i < lcap; ++i)
            g[(size_t)me * gs + kcap + i] = i < (int)pub_lm.size() ? (double)lm_gid[pub_lm[i]] : -1.0;
        farm_reserve(&tmp, &tmp_bytes, std::max<size_t>(g.size(), 1) * sizeof(double));
        HIPCHK(hipMemcpy(tmp, g.data(), g.size() * sizeof(double), hipMemcpyHostToDevice));
        farm_gather(p, tmp, gs);
        HIPCHK(hipStreamSynchronize(p->stream));
        HIPCHK(hipMemcpy(g.data(), tmp, g.size() * sizeof(double), hipMemcpyDeviceToHost));
        std::vector<int64_t> gk((size_t)R * kcap), gl((size_t)R * lcap);
        for (int r = 0; r < R; ++r) {
            for (int i = 0; i < kcap; ++i) gk[(size_t)r * kcap + i] = (int64_t)g[(size_t)r * gs + i];
            for (int i = 0; i < lcap; ++i) gl[(size_t)r * lcap + i] = (int64_t)g[(size_t)r * gs + kcap + i];
        }
        // 3. every received vertex's source offset in the exchange buffer
        const int stride = kcap * FARM_KF + 3 * lcap;
        std::vector<int> sk(p->n_kf), sl(p->n_lm);
        const int uk = p->n_kf ? lba_farm_match(me, R, kcap, gk.data(), kf_gid, kf_owner, p->n_kf, sk.data()) : 0;
        const int ul = p->n_lm ? lba_farm_match(me, R, lcap, gl.data(), lm_gid, lm_owner, p->n_lm, sl.data()) : 0;
        if (uk < 0 || ul < 0) throw ApiError{LBA_E_ARG, "farm plan: matching failed"};
        const int unmatched = uk + ul;
        std::vector<int> idx;
        for (int k : pub_kf) idx.push_back(k);
        for (int l : pub_lm) idx.push_back(p->lm_dev[l]);
        int nrk = 0, nrl = 0;
        for (int k = 0; k < p->n_kf; ++k)
            if (sk[k] >= 0) {
                const int o = sk[k] / std::max(kcap, 1), i = sk[k] - o * kcap;
                idx.push_back(k);
                idx.push_back(o * stride + i * FARM_KF);
                ++nrk;
            }
        for (int l = 0; l < p->n_lm; ++l)
            if (sl[l] >= 0) {
                if (p->lm_dev[l] < 0) continue;   // inactive here: nothing on the device to overwrite
                const int o = sl[l] / std::max(lcap, 1), i = sl[l] - o * lcap;
                idx.push_back(p->lm_dev[l]);
                idx.push_back(o * stride + kcap * FARM_KF + 3 * i);
                ++nrl;
            }
        farm_reserve(&p->f_buf, &p->f_buf_bytes, std::max<size_t>((size_t)R * stride, 1) * sizeof(double));
        farm_reserve(&p->f_idx, &p->f_idx_bytes, std::max<size_t>(idx.size(), 1) * sizeof(int));
        if (!idx.empty()) HIPCHK(hipMemcpy(p->f_idx, idx.data(), idx.size() * sizeof(int), hipMemcpyHostToDevice));
        p->f_stride = stride;
        p->f_kcap = kcap;
        p->f_npk = (int)pub_kf.size();
        p->f_npl = (int)pub_lm.size();
        p->f_nrk = nrk;
        p->f_nrl = nrl;
        p->farm_planned = true;
        if (out_counts) {
            out_counts[0] = p->f_npk; out_counts[1] = p->f_npl;
            out_counts[2] = nrk; out_counts[3] = nrl; out_counts[4] = unmatched;
        }
        return LBA_OK;
    } catch (const ApiError& e) {
        p->err = e.msg;
        return e.code;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

int lba_farm_exchange(lba_problem* p) {
    if (!p || !p->has_problem) return LBA_E_ARG;
    if (!p->farm_planned) {
        p->err = "lba_farm_exchange: no plan for this window (lba_farm_plan after lba_set_problem)";
        return LBA_E_ARG;
    }
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        const size_t S = (size_t)p->f_stride;
        double* mine = p->f_buf + (size_t)p->farm_rank * S;
        if (!p->farm_comm && p->farm_n > 1)   // the sum all-gather needs every other slot zero
            HIPCHK(hipMemsetAsync(p->f_buf, 0, (size_t)p->farm_n * S * sizeof(double), p->stream));
        const int* ik = p->f_idx;
        const int* il = ik + p->f_npk;
        const int* rk = il + p->f_npl;
        const int* rl = rk + 2 * p->f_nrk;
        launch_farm_pack(p->kst[p->cur], p->lst[p->cur], ik, p->f_npk, il, p->f_npl, p->f_kcap, mine, p->stream);
        farm_gather(p, p->f_buf, (int64_t)S);
        launch_farm_unpack(p->kst[p->cur], p->lst[p->cur], rk, p->f_nrk, rl, p->f_nrl, p->f_buf, p->stream);
        HIPCHK(hipGetLastError());
        p->gps_fresh[p->cur] = false;   // new keyframe poses need new pose samples
        p->linearized = false;
        return LBA_OK;
    } catch (const ApiError& e) {
        p->err = e.msg;
        return e.code;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

int lba_set_problem(lba_problem* p, const lba_kf* kfs, int32_t n_kf, const double* lm_xyz, int32_t n_lm,
                    const lba_obs* obs, int32_t n_obs, const lba_prior* priors, int32_t n_priors,
                    const int32_t* vel_kfs, int32_t n_vel, const lba_cam* cams, int32_t n_cam) {
    if (!p) return LBA_E_ARG;
    p->farm_planned = false;   // the plan holds device indices of the previous window
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        return set_problem(p, kfs, n_kf, lm_xyz, n_lm, obs, n_obs, priors, n_priors, vel_kfs, n_vel, cams, n_cam);
    } catch (const ApiError& e) {
        p->err = e.msg;
        release_peers(p);
        free_all(p);
        return e.code;
    } catch (const HipError& e) {
        const int rc = map_error(p, e);
        release_peers(p);
        free_all(p);
        return rc;
    }
}

int lba_optimize(lba_problem* p, int32_t iters, volatile const int32_t* stop_flag, lba_stats* out) {
    if (!p) return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        return optimize(p, iters, stop_flag, out);
    } catch (const ApiError& e) {
        p->err = e.msg;
        return e.code;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

static int get_state_buf(lba_problem* p, int buf, lba_kf* kf_out, double* lm_out) {
    if (!p || !p->has_problem) return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        std::vector<double> kst(KF_STRIDE * (size_t)std::max(p->n_kf, 1)), lst(3 * (size_t)std::max(p->n_lm_dev, 1));
        HIPCHK(hipMemcpyAsync(kst.data(), p->kst[buf], KF_STRIDE * (size_t)p->n_kf * sizeof(double),
                              hipMemcpyDeviceToHost, p->stream));
        HIPCHK(hipMemcpyAsync(lst.data(), p->lst[buf], 3 * (size_t)p->n_lm_dev * sizeof(double),
                              hipMemcpyDeviceToHost, p->stream));
        HIPCHK(hipStreamSynchronize(p->stream));
        if (kf_out)
            for (int k = 0; k < p->n_kf; ++k) {
                const double* s = kst.data() + KF_STRIDE * k;
                lba_kf& o = kf_out[k];
                for (int i = 0; i < 4; ++i) o.q[i] = s[i];
                for (int i = 0; i < 3; ++i) o.t[i] = s[4 + i];
                for (int i = 0; i < 6; ++i) o.vel[i] = s[7 + i];
                o.time = s[13];
                o.bf = s[14];
                o.fixed = p->kf_fixed[k];
                o.pad = 0;
            }
        if (lm_out)
            for (int l = 0; l < p->n_lm; ++l) {
                const int d = p->lm_dev[l];
                for (int i = 0; i < 3; ++i) lm_out[3 * (size_t)l + i] = d >= 0 ? lst[3 * (size_t)d + i] : p->lm_host[3 * (size_t)l + i];
            }
        return LBA_OK;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

int lba_get_state(lba_problem* p, lba_kf* kf_out, double* lm_out) {
    return p ? get_state_buf(p, p->cur, kf_out, lm_out) : LBA_E_ARG;
}

int lba_trial_state(lba_problem* p, lba_kf* kf_out, double* lm_out) {
    return p ? get_state_buf(p, 1 - p->cur, kf_out, lm_out) : LBA_E_ARG;
}

int lba_set_state(lba_problem* p, const lba_kf* kf_in, const double* lm_xyz) {
    if (!p || !p->has_problem) return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        if (kf_in) {
            std::vector<double> kst(KF_STRIDE * (size_t)std::max(p->n_kf, 1), 0.0);
            for (int k = 0; k < p->n_kf; ++k) {
                double* o = kst.data() + KF_STRIDE * k;
                normalize_q(kf_in[k].q, o);
                for (int i = 0; i < 3; ++i) o[4 + i] = kf_in[k].t[i];
                for (int i = 0; i < 6; ++i) o[7 + i] = kf_in[k].vel[i];
                o[13] = kf_in[k].time;
                o[14] = kf_in[k].bf;
            }
            p->gps_fresh[p->cur] = false;   // the new poses need new samples
            HIPCHK(hipMemcpyAsync(p->kst[p->cur], kst.data(), KF_STRIDE * (size_t)p->n_kf * sizeof(double),
                                  hipMemcpyHostToDevice, p->stream));
            HIPCHK(hipStreamSynchronize(p->stream));
        }
        if (lm_xyz) {
            std::vector<double> lst(3 * (size_t)std::max(p->n_lm_dev, 1));
            for (int d = 0; d < p->n_lm_dev; ++d)
                for (int i = 0; i < 3; ++i) lst[3 * (size_t)d + i] = lm_xyz[3 * (size_t)p->lm_orig[d] + i];
            for (int l = 0; l < p->n_lm; ++l)
                for (int i = 0; i < 3; ++i) p->lm_host[3 * (size_t)l + i] = lm_xyz[3 * (size_t)l + i];
            HIPCHK(hipMemcpyAsync(p->lst[p->cur], lst.data(), 3 * (size_t)p->n_lm_dev * sizeof(double),
                                  hipMemcpyHostToDevice, p->stream));
            HIPCHK(hipStreamSynchronize(p->stream));
        }
        p->linearized = false;
        return LBA_OK;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

int lba_eval(lba_problem* p, double* chi2_robust, double* obs_chi2, uint8_t* depth_ok) {
    if (!p || !p->has_problem) return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        const double chi = eval_current(p);
        if (chi2_robust) *chi2_robust = chi;
        if (obs_chi2 && p->n_obs) {
            std::vector<double> c(p->n_obs);
            HIPCHK(hipMemcpy(c.data(), p->D.ob_chi2, p->n_obs * sizeof(double), hipMemcpyDeviceToHost));
            for (int i = 0; i < p->n_obs; ++i) obs_chi2[i] = c[p->obs_dev[i]];
        }
        if (depth_ok && p->n_obs) {
            launch_depth(p->D, p->cur, p->D.depth_ok, p->stream);
            std::vector<unsigned char> h(p->n_obs);
            HIPCHK(hipMemcpyAsync(h.data(), p->D.depth_ok, p->n_obs, hipMemcpyDeviceToHost, p->stream));
            HIPCHK(hipStreamSynchronize(p->stream));
            for (int i = 0; i < p->n_obs; ++i) depth_ok[i] = h[p->obs_dev[i]];
        }
        return LBA_OK;
    } catch (const ApiError& e) {
        p->err = e.msg;
        return e.code;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

int lba_trial_chi2(lba_problem* p, double* obs_chi2) {
    if (!p || !p->has_problem || !obs_chi2) return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        HIPCHK(hipStreamSynchronize(p->stream));
        if (p->n_obs) {
            std::vector<double> c(p->n_obs);
            HIPCHK(hipMemcpy(c.data(), p->D.ob_chi2, p->n_obs * sizeof(double), hipMemcpyDeviceToHost));
            for (int i = 0; i < p->n_obs; ++i) obs_chi2[i] = c[p->obs_dev[i]];
        }
        return LBA_OK;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

int lba_linearize(lba_problem* p, double* residuals, double* H_pp, double* b, double* H_ll) {
    if (!p || !p->has_problem) return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        const DevProblem& D = p->D;
        linearize(p, residuals ? 1 : 0);
        // (no H_pp asked for: b_p alone, without the dense np x np buffer; config 4's would be 28.8 GB)
        assemble_layout(p, 0.0, H_pp ? ASM_FULL : ASM_DIAG);
        HIPCHK(hipGetLastError());
        const int np = p->np, nl = D.n_lm, npx = p->np_ext;
        std::vector<double> bp(np + 1), bl(3 * (size_t)nl + 1), hll(9 * (size_t)nl + 1), res(3 * (size_t)p->n_obs + 1);
        std::vector<double> hpp(H_pp ? (size_t)np * np + 1 : 1);
        if (H_pp && np)
            HIPCHK(hipMemcpyAsync(hpp.data(), D.Sfull, (size_t)np * np * sizeof(double), hipMemcpyDeviceToHost,
                                  p->stream));
        HIPCHK(hipMemcpyAsync(bp.data(), D.bp, np * sizeof(double), hipMemcpyDeviceToHost, p->stream));
        HIPCHK(hipMemcpyAsync(bl.data(), D.bl, 3 * (size_t)nl * sizeof(double), hipMemcpyDeviceToHost, p->stream));
        HIPCHK(hipMemcpyAsync(hll.data(), D.Hll, 9 * (size_t)nl * sizeof(double), hipMemcpyDeviceToHost, p->stream));
        if (residuals)
            HIPCHK(hipMemcpyAsync(res.data(), D.ob_res, 3 * (size_t)p->n_obs * sizeof(double), hipMemcpyDeviceToHost,
                                  p->stream));
        check_fault(p);
        const std::vector<int>& X = p->pose_ext;   // internal pose index -> caller's (extrinsics 6 wide)
        if (H_pp)
            for (int i = 0; i < np; ++i)
                for (int j = 0; j < np; ++j)
                    if (X[i] >= 0 && X[j] >= 0) H_pp[(size_t)X[i] * npx + X[j]] = hpp[(size_t)i * np + j];
        if (b) {
            for (int i = 0; i < np; ++i)
                if (X[i] >= 0) b[X[i]] = bp[i];
            int r = 0;   // landmarks in g2o order: active ones, original array order
            for (int l = 0; l < p->n_lm; ++l) {
                const int d = p->lm_dev[l];
                if (d < 0) continue;
                for (int i = 0; i < 3; ++i) b[npx + 3 * r + i] = bl[3 * (size_t)d + i];
                ++r;
            }
        }
        if (H_ll)
            for (int l = 0; l < p->n_lm; ++l) {
                const int d = p->lm_dev[l];
                for (int i = 0; i < 9; ++i) H_ll[9 * (size_t)l + i] = d >= 0 ? hll[9 * (size_t)d + i] : 0.0;
            }
        if (residuals)
            for (int i = 0; i < p->n_obs; ++i)
                for (int d = 0; d < 3; ++d) residuals[3 * (size_t)i + d] = res[3 * (size_t)p->obs_dev[i] + d];
        return npx;
    } catch (const ApiError& e) {
        p->err = e.msg;
        return e.code;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

int lba_solve_step(lba_problem* p, double lambda, double* dx) {
    if (!p || !p->has_problem) return LBA_E_ARG;
    try {
        HIPCHK(hipSetDevice(p->cfg.device));
        trial(p, lambda, false, nullptr, false);
        const int np = p->np, nl = p->D.n_lm, npx = p->np_ext;
        if (p->h_fin[3] != 0.0) {
            p->err = "reduced camera system not positive definite (factorisation status " +
                     std::to_string((long long)p->h_fin[3]) + ")";
            return LBA_E_SOLVE;
        }
        if (dx) {
            std::vector<double> x(np + 3 * (size_t)nl + 1);
            HIPCHK(hipMemcpy(x.data(), p->D.x, (np + 3 * (size_t)nl) * sizeof(double), hipMemcpyDeviceToHost));
            for (int i = 0; i < np; ++i)
                if (p->pose_ext[i] >= 0) dx[p->pose_ext[i]] = x[i];
            int r = 0;
            for (int l = 0; l < p->n_lm; ++l) {
                const int d = p->lm_dev[l];
                if (d < 0) continue;
                for (int i = 0; i < 3; ++i) dx[npx + 3 * r + i] = x[np + 3 * (size_t)d + i];
                ++r;
            }
        }
        return LBA_OK;
    } catch (const ApiError& e) {
        p->err = e.msg;
        return e.code;
    } catch (const HipError& e) {
        return map_error(p, e);
    }
}

}  // extern "C"
