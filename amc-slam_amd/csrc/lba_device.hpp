// lba_device.hpp — HBM layout of one local-BA window and the kernel launch interface.
//
// Layout (all fp64 unless noted; "device order" = landmarks sorted by the span of keyframes
// that observe them, observations grouped by landmark, so a tile of consecutive landmarks
// touches a narrow band of keyframes):
//   kf state      [n_kf][16]   q(4) t(3) vel(6) time bf pad   — two copies (current / trial)
//   lm state      [n_lm][3]                                     — two copies (current / trial)
//   observations  SoA, device order: meta(kind|cam<<4), kf_a, kf_b, pose sample, landmark,
//                 tile-local LDS row, z[3], w
//   pose samples  [n_smp][GPS_STRIDE]: per GP (prev KF, KF, observation time) the interpolated pose
//                 and the 6x24 Jacobian factor N (lba::GPSample; one per camera time stamp, not per
//                 observation), then one per KF (its pose, N = [0 | I 0]) for EdgeMono / EdgeStereo
//   Hpl           [n_hpl][12][3] one block per (non-fixed KF, heavy landmark) and per segment pair (regular
//                 tiles keep theirs in LDS; their landmarks are back-substituted in the sample space)
//   Hll, bl       [n_lm][9], [n_lm][3]
//   mslab         per (tile, pose sample) partial of M = sum rho' w J1^T J1 and g = sum rho' w J1^T e
//                 (J1 w.r.t. the sample's pose), slots sorted by sample
//   hslab/gslab   per pose sample N^T M N / -N^T g as Hpp blocks (aa, ab, bb) / b_p pieces, and per
//                 prior / velocity edge, each block stored at a slot sorted by its target upper block
//   sslab/gpslab  per (tile, KF pair) Schur partials V(k1) Hpl(k2)^T and per (tile, KF) rhs
//                 partials, target-sorted likewise
//   S, Lm         [npad][npad] dense reduced camera system (lower) and its Cholesky factor; npad =
//                 np rounded up to CHOL_NB with an identity tail, so every Cholesky panel is full
#pragma once

#include <hip/hip_runtime.h>

namespace lba {

constexpr int KF_STRIDE = 16;
constexpr int CAMD_STRIDE = 88;     // Rcb(9) tcb(3) fx fy cx cy, extrinsic factor Ad(Tbc) (lba::cam_record)
constexpr int SEG_STRIDE = 8;      // seg_slot ints per slab entry (see DevProblem::seg_slot)
constexpr int GSEG_STRIDE = 3;     // seg_gslot ints per slab entry
constexpr int KFP_STRIDE = 12;      // Rwb(9) twb(3)

// tile limits (one workgroup of TILE_OBS threads per tile)
constexpr int TILE_OBS = 128;
// in-launch hand-off flags (k_update's producers, k_exp_asm's expansions): one per 128-byte line, so the polls of
// different producers' flags do not queue on one line
#ifndef LBA_FLAG_STRIDE
#define LBA_FLAG_STRIDE 32
#endif
constexpr int FLAG_STRIDE = LBA_FLAG_STRIDE;   // ints
constexpr int CF_TDBG_STRIDE = 8 + 2 * 16;     // diagnostics: u64 per k_chol_flow factor task
constexpr int UPD_BLOCK_KFS = 64;   // keyframes per KF-block workgroup of k_update (its UPD_THREADS)
constexpr int TILE_ROWS = 288;
constexpr int TILE_PAIRS = 128;
constexpr int TILE_LMS = 64;
constexpr int TILE_KF = 16;
constexpr int ROW_STRIDE = 10;      // LDS Jacobian row: J1(6) e(1) Jp(3) (J1: w.r.t. the pose sample)
constexpr int G_STRIDE = 18;        // per observation: G = rho' w sum_rows J1^T Jp (6 x 3, row-major)
constexpr int SM_STRIDE = 27;       // per (tile, sample) partial: M = sum rho' w J1^T J1 (21, upper
                                    // row-major) and g = sum rho' w J1^T e (6)
// slot pitches of the partial slabs in doubles: every slot fills whole 128-byte lines of its own, so a slot handed from
// its producer to its consumer inside one launch (k_exp_asm's gslab pieces) shares no line with another target's
// slots (hslab / sslab slots are 144 doubles = 9 lines already)
constexpr int MS_PITCH = 32;        // mslab: 27 used
constexpr int GS_PITCH = 16;        // gslab / gpslab: 12 used
constexpr int TILE_SMP = 64;        // pose samples per tile (k_linearize stages their row runs)
constexpr int TILE_PROWS = 2 * TILE_OBS;    // pair entry-list entries per tile (each obs feeds <= 2 pairs)
constexpr int TILE_SENT = TILE_KF * (TILE_KF + 1) / 2;   // KF-pair Schur entries per tile

constexpr int CHOL_NB = 32;         // Cholesky panel / tile width
constexpr int CF_DENSE_MAX_NP = 192;   // panels up to which the L^-1-tile solve is allowed (np 6144)
constexpr int CF_AUTO_BAND_NP = 64;    // above this many panels the substitution solve is the default
                                       // (measured crossover ~65 panels, profiles/r01zr_solve_sweep.txt)
#ifndef LBA_RED_GROUPS
#define LBA_RED_GROUPS 4
#endif
constexpr int RED_GROUPS = LBA_RED_GROUPS;   // reduction kernels: 4 groups x 144 threads

// Levenberg-Marquardt controller of a queued optimisation (lba_host.hip: optimize_queued).  The host
// enqueues whole trials without waiting for their outcome; k_finalize applies g2o's acceptance rule
// (optimization_algorithm_levenberg.cpp:56-140) to this record, and the kernels of the next trial read
// from it which state buffer is current, the damping, and whether they run at all.
struct LMCtl {
    double lambda, ni;
    double cur_chi, ini_chi;   // currentChi / iniChi of the iteration in progress
    double last_chi;           // chi2 of the last evaluated trial state (g2o's activeRobustChi2)
    double chi0;               // chi2 of the starting state (lba_stats.chi2_initial)
    int cur;                   // state buffer holding the current estimate (the other one: trial)
    int qmax;                  // trials of the iteration in progress
    int it, iters;             // iterations completed / requested
    int done;                  // 1: every further kernel of the queue is a no-op
    int need_lin;              // 1: the next trial starts a new iteration (relinearise first)
    int nbad, trials, failures, result;
    int max_trials, early_stop;
    int slot;                  // trials finalised (queue position)
    int chi0_lin;              // 1: chi0 is still to be taken from the first trial (its chi2 at the linearisation point)
};
constexpr int LMCTL_DOUBLES = sizeof(LMCtl) / sizeof(double);
static_assert(sizeof(LMCtl) % sizeof(double) == 0, "LMCtl mirrors into a double array");

// state-buffer selection of a launch: a fixed buffer (host-driven trials), or the controller's
// current / trial buffer (queued trials)
enum { SEL_CUR = 2, SEL_NEXT = 3 };
// launch gating in a queued optimisation: run always, unless the queue is done, or only when the
// trial starts a new iteration
enum { GATE_NONE = 0, GATE_TRIAL = 1, GATE_LIN = 2 };
// lambda argument: take the controller's damping.  A NaN, so that every real damping a caller passes
// (lba_solve_step at any lambda, negative ones included: BlockSolver::setLambda takes any value) is used as is
constexpr double LAMBDA_CTL = __builtin_nan("");

// fault codes (DevProblem::fault): which bounded wait timed out
enum { FAULT_FLOW = 1, FAULT_EXP = 2, FAULT_UPD = 4 };
constexpr int RED_FAULT_BITS = 3;
constexpr int RED_N = 4 + RED_FAULT_BITS;   // doubles of DevProblem::red4

struct DevProblem {
    int n_kf, n_lm, n_obs, n_gp, n_pairs, n_tiles, n_pb, np, n_prior, n_vel, n_cam;
    int npad;               // np rounded up to CHOL_NB: leading dimension of S / Lm (identity tail)
    int n_entries, n_sentries, n_ublocks;
    // slab and table extents (LBA_DEBUG_BOUNDS builds check every indexed write against them)
    int n_mslots, n_hslots, n_gslots, n_sslots, n_gpslots, n_chi, n_lm_all;
    // observations (device order)
    const int* ob_meta;
    const int* ob_kfa;
    const int* ob_kfb;
    const int* ob_smp;      // pose sample (lba::GPSample): GP sample, or n_gps + kf_b for EdgeMono/Stereo
    const int* ob_lm;
    const int* ob_row;      // tile-local LDS row | (regular tiles) tile-local pose sample << 16
    const double* ob_z;     // [n_obs][3]
    const double* ob_w;
    // keyframes
    const int* kf_hidx;
    const int* gp_kfa;      // per GP pair (prev KF, KF)
    const int* gp_kfb;
    const int* gp_hab;      // per GP pair: KF a, KF b, their pose blocks (-1: fixed)
    const int* gp_s0;       // [n_gp + 1] the pair's pose samples (contiguous)
    const double* gps_t;    // per GP sample: observation time
    int n_gps;              // GP samples; samples n_gps .. n_gps + n_kf - 1 are the KF poses (N = [0 | I 0])
    int n_smp;              // n_gps + n_kf
    double* camdb[2];       // [n_cam][CAMD_STRIDE] camera records of state buffer 0 / 1 (they differ only for
                            // cameras with a free extrinsic: k_update rewrites those from the trial state)
    const int* kf_cam;      // [n_kf] camera whose extrinsic a KF slot holds, -1 for keyframes
    int n_kf_user;          // KF slots n_kf_user .. n_kf - 1 are the free extrinsics (pose blocks after the KFs)
    int n_eprior;           // EdgeExtrinsicPrior edges (one per free extrinsic), slab entries after the velocity edges
    const int* ep_kf;       // per extrinsic prior: its KF slot
    const double* ep_data;  // per extrinsic prior: [16] R_ini^-1 quaternion (4), information (9)
    // tiles: [0, n_stiles) regular tiles (linearised and eliminated by k_lin_schur), then
    // [n_stiles, n_tiles) the segments of the heavy landmarks (linearised like tiles; their Hll / bl
    // partials go to landmark slots n_lm + segment, their Hpl partials to segment pairs n_pairs ..)
    int n_stiles;
    // heavy landmarks (too many observations / keyframes for one tile; device indices n_lm - n_heavy ..
    // n_lm - 1): one k_expand work item each merges the segments' partials and eliminates the landmark
    int n_heavy;
    const int* hv_lm;       // [n_heavy] device landmark
    const int* hv_seg0;     // [n_heavy + 1] segments (landmark slots n_lm + s)
    const int* hv_hp0;      // [n_heavy + 1] heavy pairs: hp = hv_hp0[h] + i is canonical pair lm_pair0[lm] + i
    const int* hp_src0;     // [n_hpairs + 1] CSR into hp_src: the segment pairs summing into a heavy pair
    const int* hp_src;
    const int* hp_gslot;    // [n_hpairs] gpslab slot of the heavy pair's rhs partial
    const int* hv_ss0;      // [n_heavy + 1] sslab slots of the landmark's KF-pair blocks (a <= b, a-major)
    const int* hv_sslot;
    double* Vh;             // [n_hpairs][36] V = Hpl Dinv of the heavy pairs (scratch)
    const int* pair_lk;     // per pair of a regular tile: tile-local KF | tile-local landmark << 8
    const int* tile_obs0;
    const int* tile_nobs;
    const int* tile_lm0;
    const int* tile_nlm;
    const int* tile_pair0;
    const int* tile_npair;
    const int* tile_smp0;   // per tile: first tile-sample record / count
    const int* tile_nsmp;
    const int* tsm_meta;    // per tile sample: row0 | nrows << 16 (tile-local LDS rows), mslab slot
    const int* tile_sent0;
    const int* tile_nsent;
    const int* tile_kf0;
    const int* tile_nkf;
    const int* tile_perm;        // k_lin_schur workgroup -> tile (longest first)
    const int* tkf_list;    // tile KF unions (pose block indices)
    const int* sent_l1;     // per Schur entry: tile-local KF index of k1 / k2
    const int* sent_l2;
    // pairs / landmarks
    const int* pair_lm;
    const int* pair_kf;     // pose block index
    const int* pair_r0;     // CSR into pair_rows: tile-local observation | side << 16 (0: KF a, 1: KF b)
    const int* pair_rows;
    const int* lm_r0;       // CSR into lm_rows: tile-local rows
    const int* lm_rows;
    const int* lm_pair0;    // [n_lm + 1] landmark -> pairs
    // k_update's back-substitution of the regular tiles' landmarks in the sample space (no Hpl): per tile
    // sample its pose sample (tsm_smp) and that sample's pose blocks of KF a / KF b / extrinsic (-1: fixed
    // or none) and the camera of the extrinsic factor (tsm_blk, 4 ints), per device landmark its
    // observations (lm_obs0, [n_lm + 1])
    const int* tsm_smp;
    const int* tsm_blk;
    const int* lm_obs0;
    // Hpl is stored only for the heavy landmarks' pairs: pair index q lives at slot q - hpl_base
    // (canonical heavy pairs, then the segment pairs); n_hpl slots
    int hpl_base, n_hpl;
    // partial-sum slabs are sorted by their reduction target, so every reduction below reads
    // one contiguous range (coalesced) instead of chasing a source list
    const int* seg_slot;    // per slab entry (pose samples, motion priors, velocity edges, extrinsic priors):
                            //   SEG_STRIDE ints: aa, ab, bb slot in hslab (-1 = none), ab transposed flag,
                            //   ae, be, ee slot (a sample's extrinsic block e), camera of e
    const int* seg_gslot;   // per slab entry: ga, gb, ge slot in gslab (-1 = none)
    const int* asm_list;    // upper blocks inside the structural pattern of S (diagonal + any source)
    int n_asm;
    int n_ztiles;           // tiles of L (S and L are stored as these tiles), zeroed before each assembly
    const int* hs0;         // [n_ublocks + 1] hslab range per upper block
    const int* gs0;         // [n_pb + 1] gslab range per pose block
    const int* ub_i;        // per upper block: block row / col
    const int* ub_j;
    const int* sslot;       // per Schur entry: slot in sslab
    const int* ss0;         // [n_ublocks + 1] sslab range per upper block
    const int* tkf_gslot;   // per tile KF: slot in gpslab (Schur g partials)
    const int* gps0;        // [n_pb + 1] gpslab range per pose block
    // motion-prior / velocity edges
    const int* pri_a;
    const int* pri_b;
    const int* vel_kf;
    int pri_entry0;         // slab entry index of prior 0 (velocity edges follow); samples are 0..n_smp-1
    const int* ms0;         // [n_smp + 1] mslab range per sample
    double qcinv[36];
    double huber_mono, huber_stereo, huber_prior;
    // work buffers
    double* gpsb[2];        // [n_smp][GPS_STRIDE] pose samples (Rwb twb N, lba::GPSample) of state buffer 0 / 1
    double* mslab;          // [n_mslots][MS_PITCH] per (tile, sample) M / g partials, sample-sorted
    double* kfp_pose;       // [n_kf][KFP_STRIDE] Rwb twb (same prefix as a sample)
    double* hslab;          // [n_hslots][144] Hpp partial blocks, target-sorted
    double* gslab;          // [n_gslots][GS_PITCH] b_p partials, target-sorted
    double* sslab;          // [n_sslots][144] Schur partial blocks, target-sorted
    double* gpslab;         // [n_gpslots][GS_PITCH] Schur rhs partials, target-sorted
    double* Lm;             // Cholesky factor, the same tiles as S (lower)
    // dense solve in the factorisation (nested-dissection) order of the panels: position = ppos[natural],
    // natural = pnat[position]; pfirst = envelope of the permuted matrix
    const int* ppos;
    const int* pnat;
    // rows: natural -> factorisation order (the block ordering of the keyframes, then the panel
    // permutation of the dissection) and back; [npad], the identity on the padding rows
    const int* rpos;
    const int* rnat;
    // dataflow factorisation (k_chol_flow): tasks, tile ids, hand-off flags, ticket counter
    const int* cf_tasks;    // j | kind << 24 | lookahead << 28
    const int* cf_task_i;   // i
    const int* cf_task_t;   // [5] tile ids a factor task holds: (j,j), (i,j), (k,k), (j,k), (i,k) (-1: none)
    int cf_ntasks;
    const int* cf_rowptr;   // tiles of L by row (factorisation order): row i's tiles cf_rowptr[i] .. [i + 1]
    const int* cf_cols;     //   their columns, ascending (tile id = index)
    double* cf_linv;        // [npad][npad] L^-1 tiles (k_chol_flow)
    int* cf_ivready;        // per lower tile i (i + 1) / 2 + j
    const int* cf_pl0;
    const int* cf_plist;
    const int* cf_plist_t;  // [3] tile ids per update / term entry
    int* cf_lready;
    int* cf_dready;
    int* cf_fready;
    int* cf_zready;
    double* cf_zv;          // [NP][NP][CHOL_NB] shares Linv(i, k) b_k of the forward solve
    unsigned long long* cf_head;
    int* cf_abort;
    int cf_band;            // 1: solve by substitution tasks (no L^-1 tiles, large systems)
    unsigned long long* cf_xg;   // band solve: x in factorisation order as {epoch, half} granules (back tasks)
    double* LinvT;          // [npad / CHOL_NB][CHOL_NB][CHOL_NB] inverse diagonal blocks L_bb^-T (row-major)
    double* Hpl;
    double* Hll;
    double* bl;
    double* Dinv;
    double* S;              // [n_ztiles][32][32] the reduced system in factorisation order, stored as the tiles
                            // of L (cf_rowptr / cf_cols: the symbolic factorisation), padding: identity
    double* Sfull;          // [np][np] natural order, both triangles (ASM_FULL: lba_linearize), allocated on use
    double* Sdiag;          // [np] natural diagonal of H_pp (ASM_DIAG: computeLambdaInit)
    double* bp;             // [np]
    double* bS;             // [npad] reduced right-hand side b_p - sum Hpl Dinv bl (factorisation order)
    double* xsol;           // [npad] solution (natural order)
    double* yv;             // [np] forward-substituted rhs
    double* x;              // [np + 3 n_lm]
    double* chi_lin;        // [n_tiles + n_prior + n_vel + n_eprior]
    double* chi_eval;       // [n_tiles + n_prior + n_vel + n_eprior]
    double* scale_part;     // [n_upd_blocks]
    int n_upd_blocks;
    // fused trial evaluation (k_update with eval = 1): the regular tiles evaluate their observations at the trial
    // state once the pose samples are made, extra workgroups the motion-prior / velocity edges (no heavy landmarks,
    // no free extrinsics); upd_flag [n_gp + KF blocks]: a producer's epoch once its samples / states are stored,
    // smp_prod [n_smp]: the producer of each pose sample (its GP pair, or the KF block of a KF pose sample)
    int fuse_eval;
    // the fp32-residual option (LBA_FLAG_F32_RESIDUAL): the kernels' per-observation projection, residuals and
    // Jacobian rows in fp32, every sum in fp64 (k_lin_schur / k_update / k_eval's <true> instantiations)
    int f32res;
    int* upd_flag;
    const int* smp_prod;
    // fused expansion + assembly (k_exp_asm; no heavy landmarks, not partitioned): exp_flag [n_smp] a pose sample's
    // epoch once its Hpp / b_p pieces are stored; hs_prod [n_hslots] / gs_prod [n_gslots] the sample that writes
    // each slot (< 0: an edge item of k_lin_schur)
    int fuse_asm;
    int* exp_flag;
    const int* hs_prod;
    const int* gs_prod;
    double* kbuf[2];        // kf state buffers [n_kf][KF_STRIDE] (current / trial, see LMCtl::cur)
    double* lbuf[2];        // landmark state buffers [n_lm][3]
    LMCtl* ctl;             // queued-optimisation controller
    int* hlog;              // host-mapped [HLOG_CAP]: per queued trial, 1 if it relinearised
    int* info;              // [1] factorisation status
    // [1] a bounded in-launch wait that gave up (FAULT_*, never expected): the data it waited for may be stale, so
    // k_finalize publishes it (hfin[5]) and the host fails the call with LBA_E_TIMEOUT instead of using the results
    int* fault;
    double* fin;            // [4] chi_lin, chi_eval, scale, info
    double* hfin;           // host-mapped coherent [4] copy of fin + [4] sequence number (as bits)
    double* ob_chi2;        // [n_obs]
    double* ob_res;         // [n_obs][3]
    unsigned char* depth_ok;   // [n_obs] isDepthPositive flags (lba_eval)
    // partitioned global BA (lba_set_partition): this rank holds a subset of the landmarks; the
    // reduced system, b_p and the trial sums are summed over the ranks by the caller's all-reduce
    int part_rank, part_n;  // rank / ranks (part_n 0: not partitioned)
    // natural row r of the reduced system: the rank whose subtree of the distributed factorisation holds it,
    // -1 for rows every rank holds (the top of the split, every row when the solve is replicated); the
    // damping, the padding identity and the computeScale terms of a row are added on its owner (rank 0 for -1)
    const int* row_own;
    // distributed factorisation (LBA_FLAG_SUBTREE_SOLVE): k_chol_flow runs twice per trial, the subtrees'
    // tasks (cf_tasks ...) then, after the all-reduce of the top tiles (top_tiles) and of bS / b_p, the top's
    // tasks and the back substitution (cf_tasks2 ...)
    int cf_split;
    const int* cf_tasks2;
    const int* cf_task_i2;
    const int* cf_task_t2;
    const int* cf_pl02;
    const int* cf_plist2;
    const int* cf_plist_t2;
    int cf_ntasks2;
    const int* top_tiles;   // tiles of L in the top columns (packed into env_buf ahead of bS / b_p)
    int n_top_tiles;
    double* red4;           // [RED_N] trial sums of this rank, the factorisation status, then the fault word's bits,
                            // all-reduced before k_finalize reads them
    double* env_buf;        // [n_env] (cf_split: the top tiles,) bS [npad], then b_p [np] (all-reduce buffer; replicated
                            // solve: S is all-reduced in place)
    long long n_env;
    // diagnostics (LBA_PHASE_TIMING=<file>): per-workgroup clock64() stamps at phase boundaries
    unsigned long long* tdbg_lin;     // [n_tiles][16] k_linearize
    unsigned long long* tdbg_schur;   // [n_tiles][16] k_schur
    unsigned long long* tdbg_chol;    // [npad / CHOL_NB][16] k_chol_flow panel tasks
    unsigned long long* tdbg_cf;      // [4096][CF_TDBG_STRIDE] k_chol_flow factor tasks: stamps, i, j; then per update-list
                                      // entry (the first 16): its end stamp and (panel | waited << 24)
    unsigned long long* tdbg_bs;      // [npad / CHOL_NB][16] k_chol_flow L^-1 tasks of the last rows
};

// launchers (lba_kernels.hip).  sel: state buffer (0 / 1, or SEL_CUR / SEL_NEXT from the controller);
// gate: GATE_*; lambda: the damping, or LAMBDA_CTL
constexpr int HLOG_CAP = 4096;
void launch_gp_prep(const DevProblem& P, int sel, int jac, int gate, hipStream_t s);
// e0 / e1 (optional): timing events attached to the k_linearize dispatch itself
// edges: also the motion-prior / velocity / extrinsic-prior quadratic forms of launch_prior_lin, as extra
// workgroups after the tiles (the pose samples' part then comes with launch_schur(psel, pgate))
// linearisation of every tile (+ with LS_SCHUR the landmark elimination into the S / rhs partials), the
// motion-prior / velocity / extrinsic-prior quadratic forms with LS_EDGES, residuals out with LS_RES;
// lambda: the damping (LAMBDA_CTL: the controller's); e0 / e1 (optional): events on the dispatch itself
enum { LS_SCHUR = 1, LS_EDGES = 2, LS_RES = 4 };
void launch_lin_schur(const DevProblem& P, int sel, int gate, double lambda, int mode, hipStream_t s,
                      hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
// pose-sample expansion (N^T M N into the Hpp / b_p slabs) and the heavy landmarks (merge of their segments;
// with schur also their elimination)
void launch_expand(const DevProblem& P, int sel, int gate, double lambda, int schur, hipStream_t s);
enum { ASM_SCHUR = 1, ASM_FULL = 2, ASM_DIAG = 4 };
void launch_assemble(const DevProblem& P, double lambda, int flags, int gate, hipStream_t s);
// k_expand (schur) + k_assemble (ASM_SCHUR) of a trial in one launch (P.fuse_asm); epoch: one more than the last
void launch_exp_asm(const DevProblem& P, int sel, int gate, double lambda, unsigned epoch, hipStream_t s);
void launch_cholesky_solve(const DevProblem& P, int gate, unsigned epoch, hipStream_t s, hipEvent_t e0 = nullptr,
                           hipEvent_t e1 = nullptr);
// the step + trial state + the trial state's pose samples (jac: with their Jacobian factors)
// eval: with P.fuse_eval, also the trial state's errors (k_eval's chi_eval / ob_chi2), no k_eval launch needed;
// update_grid: its workgroups; update_resident_blocks: k_update workgroups resident at once on the device
int update_grid(const DevProblem& P, int eval);
int update_resident_blocks(int device);
void launch_update(const DevProblem& P, double lambda, int sel, int gate, int jac, hipStream_t s, int eval = 0,
                   unsigned epoch = 0);
// partitioned mode: this rank's trial sums into red4; envelope of S + bS + b_p into / out of env_buf
void launch_partials(const DevProblem& P, hipStream_t s);
void launch_env_pack(const DevProblem& P, int unpack, int gate, hipStream_t s);
// distributed factorisation: part 0 (the rank's subtrees and its contributions to the top) / part 1 (the top
// and the back substitution) of k_chol_flow (same epoch for both)
void launch_cholesky_part(const DevProblem& P, int part, unsigned epoch, hipStream_t s, hipEvent_t e0 = nullptr,
                          hipEvent_t e1 = nullptr);
enum { FIN_NONE = -1, FIN_HOST = 0, FIN_QUEUED = 1, FIN_QUEUED_PUBLISH = 2 };
void launch_finalize(const DevProblem& P, unsigned long long seq, int mode, hipStream_t s);
// zero n device ranges (pairs: address, 4-byte words) in one launch (lba_set_problem's fresh buffers)
void launch_zero_ranges(const unsigned long long* ranges, int n, size_t words, hipStream_t s);
// residual evaluation of a state, then (mode != FIN_NONE) the trial summary (k_finalize)
void launch_eval(const DevProblem& P, int sel, int gate, unsigned long long seq, int mode, hipStream_t s);
void launch_ctl_init(const DevProblem& P, const LMCtl& c, hipStream_t s);
void launch_lambda_init(const DevProblem& P, double tau, hipStream_t s);
void launch_depth(const DevProblem& P, int sel, unsigned char* ok, hipStream_t s);

// window farm: a published keyframe is its q (4), t (3) and velocity (6), the prefix of its state record
constexpr int FARM_KF = 13;
void launch_farm_pack(const double* kst, const double* lst, const int* pub_kf, int npk, const int* pub_lm, int npl,
                      int kcap, double* out, hipStream_t s);
void launch_farm_unpack(double* kst, double* lst, const int* rkf, int nrk, const int* rlm, int nrl, const double* buf,
                        hipStream_t s);

constexpr int GPS_STRIDE = 156;     // doubles in lba::GPSample (static_assert in lba_kernels.hip)

}  // namespace lba
