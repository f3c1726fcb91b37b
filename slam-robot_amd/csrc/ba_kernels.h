// ba_kernels.h — data layout shared by the bundle-adjustment kernels and their host driver.
//
// HBM layout (all fp64, structure-of-arrays, points in "first free block" order so that a chunk of
// consecutive points touches a narrow window of camera blocks — the co-visibility band of a sliding
// window BA):
//   q[2][4F], t[2][3F], X[2][4P]   parameter state, two slots (current / candidate), switched by LmState::cur
//   obs_pt[2M], obs_frame[M]       observations, CSR by point (poff[P+1])
//   J[2][M/64][12][64] (double2)   corrected, unscaled residual + Jacobian per observation, element pairs
//                                  (r~ 2 | Jc 2x6 [rot_local 3, t 3] | Jp 2x4 | pad 2), one slot per parameter
//                                  slot: the linearization at x[cur], and the one k_update_lin forms at the
//                                  candidate x[cur ^ 1] (it becomes current when the step is accepted)
//   V[2][P][10], g[2][P][4]        point normal-equation blocks (upper 4x4) and gradient, slotted like J
//   Vinv[P][10], tp[P][4]          damped, scaled inverse and V^-1 g~ (per LM iteration)
//   cam_slab / S_slab              per-chunk partial camera blocks / per-segment Schur tiles (deterministic
//                                  reduce)
//   S[n][n], xc[n]                 dense reduced camera system (upper blocks), n = 6 * free frames, and
//                                  its rhs, contiguous (one all-reduce over landmark shards)
#ifndef SG_BA_KERNELS_H_
#define SG_BA_KERNELS_H_

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sg {

constexpr int kCamV = 27;           // per camera block: upper(Jc^T Jc) 21 + Jc^T r 6
// Observation record (ba_device.h jidx2): r~ 2 | rotation Jacobian 2x3 | point Jacobian 2x4 = 16 doubles; the
// translation Jacobian is not stored (J~t = -X.w J~p[:, 0:3], jc_trans)
constexpr int kJPairs = 8;
constexpr int kJStride = 2 * kJPairs;
constexpr int kNScal = 16;          // per-chunk scalar slots
constexpr int kCholThreads = 512;
constexpr int kCholNb = 16;

enum ScalSlot {
  kCost = 0, kFail, kFixed, kFixedFail, kXnorm2, kGmax, kLinFail, kModel, kCandCost, kCandFail, kStep2,
  kCandX2
};

// Packed per-observation facts (device order), so that a sweep lane's loads depend only on its own
// observation record: camera block + 1 (0: frame not free) in bits 0-15, camera in bits 16-23, then the
// frame's rotation / translation freedom, the point's freedom and the fixed flag (all blocks constant).
constexpr int kMetaCamShift = 16;
constexpr int kMetaRot = 1 << 24, kMetaTrans = 1 << 25, kMetaPfree = 1 << 26, kMetaFixed = 1 << 27;
__host__ __device__ __forceinline__ int meta_block(int m) { return (m & 0xffff) - 1; }
__host__ __device__ __forceinline__ int meta_cam(int m) { return (m >> kMetaCamShift) & 0xff; }

// Exchange-buffer scalar slots appended after the camera blocks.
enum CamX { kXCost = 0, kXFail, kXFixed, kXFixedFail, kXXnorm2, kXNum };
enum UpdX { kUModel = 0, kUCandCost, kUCandFail, kUStep2, kUCandX2, kULinFail, kUTimeout, kUNum };
// kCTimeout: cross-wave / cross-workgroup hand-offs of the tiled Cholesky that hit their spin limit (the
// step is then not trusted: the solve ends with SG_DEVICE_TIMEOUT, see decide_step)
enum CholX { kCStep2 = 0, kCCandX2, kCModel, kCCandCost, kCFail, kCTimeout, kCNum };


// k_schur work decomposition (see ba_solver.hip): a segment is a run of consecutive points (device order)
// whose camera columns fit a window of <= kSchurTW 16-column tiles of S, one workgroup (kSchurCWaves waves holding
// the window's upper tiles and rhs rows in MFMA accumulators, a point wave, kSchurCellWaves building the
// operand tiles); it streams through
// LDS in batches of <= kSchurBatchPts points whose operand tiles (64 doubles each) fit kSchurXCap.  The cells
// of a point (one per block of its span) carry its observations.  A point spanning more than kSegNbMax blocks
// is a WideSeg of its own (observation pairs, global atomics).
#ifndef SG_SEG_NB
#define SG_SEG_NB 24   // widest point of a segment, in blocks (6 * 24 + 14 <= 16 * kSchurTW columns)
#endif
constexpr int kSegNbMax = SG_SEG_NB;
static_assert(kSegNbMax <= 24, "cells of a batch: kSchurBatchCells");
constexpr int kSchurCellWaves = 3;   // operand-tile waves (a batch has <= 64 kSchurCellWaves cells)
#ifndef SG_SCHUR_CW
#define SG_SCHUR_CW 4
#endif
constexpr int kSchurCWaves = SG_SCHUR_CW;   // MFMA waves (4: one per SIMD; 8: two); a point wave between the groups
constexpr int kSchurWaves = kSchurCellWaves + 1 + kSchurCWaves;
constexpr int kSchurThreads = 64 * kSchurWaves;
#ifndef SG_SCHUR_TW
#define SG_SCHUR_TW 10   // window width in tiles (variant builds: tools/build_variant.sh)
#endif
constexpr int kSchurTW = SG_SCHUR_TW;
constexpr int kSchurTiles = kSchurTW * (kSchurTW + 1) / 2;
constexpr int kSchurAug = kSchurTiles + kSchurTW;   // window tiles + one rhs tile per tile row
constexpr int kSchurTPW = (kSchurAug + kSchurCWaves - 1) / kSchurCWaves;   // accumulator tiles per wave
constexpr int kSchurXCap = 112 * 64;   // operand tiles (64 doubles each) per batch buffer
#ifndef SG_SCHUR_BATCH
#define SG_SCHUR_BATCH 32
#endif
constexpr int kSchurBatchPts = SG_SCHUR_BATCH;   // <= 64: a batch's point table is one point per lane
constexpr int kSchurBatchCells = kSchurBatchPts * 24;   // cells of a batch (spans <= kSegNbMax)
static_assert(6 * kSegNbMax + 14 <= 16 * kSchurTW, "a widest point must fit the tile window");
struct SchurSeg {
  int32_t p0, p1;       // point range
  int32_t b_lo, nb;     // blocks the points observe: rhs partial [b_lo, b_lo + nb)
  int32_t s_off;        // S_slab offset: ntw (ntw + 1) / 2 row-major 16x16 tiles, then 6 nb rhs entries
  int32_t t0, ntw;      // window: tile columns [t0, t0 + ntw) of S
  int32_t bt0, bt1;     // batches
  int32_t pad;
};
struct SchurBatch {
  int32_t p0, p1;       // points
  int32_t c0, c1;       // cells
};
struct WideSeg {
  int32_t p;            // the point
  int32_t pair_lo, pair_hi;
  int32_t pad;
};

// k_linearize work decomposition: a chunk (one single-wave workgroup) is a run of consecutive points whose
// camera blocks fit one window of <= kLinNbMax blocks, split into rounds of <= kLinObs observations and
// <= kLinPts points that hold whole points (one observation per lane).  A point with more observations, or
// spanning more blocks, is a "wide" chunk of its own: rounds are pieces of it and its camera terms go to
// global atomics.  A chunk's workgroup has one or two waves (BaSolver::lin_waves_, fixed at load: two when the
// grid would leave SIMDs idle): wave w takes rounds r0 + w, r0 + w + 2, ... into LDS accumulators of its own,
// summed in wave order at the end (a wide chunk runs on wave 0).
constexpr int kLinThreads = 64;   // lanes of one wave (one observation per lane)
constexpr int kLinObs = 64;
constexpr int kLinPts = 16;
constexpr int kLinNbMax = 24;
constexpr int kLinMaxRounds = 4;   // measured best at 130k and 1.6M observations
struct LinRound {
  int32_t o0, o1;     // observation range
  int32_t p0, p1;     // points (whole points; every piece of a wide point names it)
};
struct LinChunk {
  int32_t r0, r1;     // round range
  int32_t b_lo, nb;   // camera window [b_lo, b_lo + nb) (nb = 0: no camera terms in LDS)
  int32_t cam_off;    // offset of this chunk's camera partials in cam_slab (doubles)
  int32_t wide;       // one point: camera terms by global atomics, point block reduced over the workgroup
  int32_t p0, p1;
  int32_t u0;         // its first k_point_update work unit (one per round; one for a wide chunk)
};

// Concurrency contract.  Two launches store the whole LmState from one thread while other workgroups of the
// SAME launch read it: k_cam_reduce mode 2 (workgroup NB+1 takes the decision while workgroups 0..NB read
// `done` and `spec_slot`) and k_schur with fin (workgroup 0 runs the finalize pass while the segments read `cur`,
// `done`, `reuse_diag` and `radius`).  Within those launches the writer may change only `done` (a reader that
// sees the old value does the work the next launch would discard anyway), `accepted`, the counters and the cost
// bookkeeping; `cur`, `spec_slot`, `reuse_diag` and `radius` are changed only by launches in which nothing else
// reads them (the decision of k_cam_reduce mode 2 flips `cur` / sets `radius` for the NEXT launch, and its
// readers in that launch read `done` / `spec_slot` only).  An edit that breaks this must hand the readers their
// fields through a separate word written by an earlier launch.  Those launches store through lm_store_shared
// (ba_lm.h), which writes only the fields listed here, so a stray edit of a read field cannot reach memory.
struct LmState {
  // options (copied from sg_solver_options)
  int32_t max_iter, max_invalid, disable_term, jacobi;
  int32_t always_lin, pad1;   // benchmark: linearize after a rejected step too (sg_solver_options.always_linearize)
  double ftol, gtol, ptol, min_rel_dec, max_radius, min_radius, min_diag, max_diag;
  // minimizer state
  int32_t cur, need_lin, first, done;
  int32_t termination, ok, pushed, lm_iters;
  int32_t n_succ, n_unsucc, n_invalid, consecutive_invalid;
  int32_t reuse_diag, sync_timeouts;   // sync_timeouts: Cholesky hand-off time-outs seen (kCTimeout)
  // speculative chain: the slot k_update_lin linearized the candidate into (written by k_update_lin only), and
  // whether the last decision accepted a step whose candidate camera blocks (xchg_cand) are still to be taken
  int32_t spec_slot, accepted;
  double radius, decrease_factor;
  double cost, fixed_cost, initial_cost, x_norm, abs_gtol, min_pushed_cost;
  double last_model, last_new_cost, last_rel_decrease, last_step_norm;
};

// Kernel argument bundle (passed by value through the kernarg segment).
struct Dev {
  LmState* st;
  // cameras / frames
  double* k[2];                  // intrinsics [ncam][7], two slots (current / candidate) like q, t, X
  double* q[2];
  double* t[2];
  const int32_t* frame_cam;
  const int32_t* frame_block;
  const uint8_t* rot_free;
  const uint8_t* trans_free;
  int32_t F, NB, n;
  // points / observations
  double* X[2];
  const uint8_t* pfree;
  const int32_t* poff;
  int32_t P, M;
  const double* obs_pt;
  const int32_t* obs_frame;
  const uint8_t* obs_fixed;
  double b, inv_b;               // Cauchy(range): b = range^2
  // FrameDistance
  int32_t D;
  const int32_t* fd_a;           // problem frame index
  const int32_t* fd_b;
  const int32_t* fd_boff;        // per block CSR of incident FD residuals (entry = 2*d + side)
  const int32_t* fd_bidx;
  double fd_target, fd_b2, fd_inv_b2;
  double* fd_r;                  // [D] corrected residual
  double* fd_J;                  // [D][6] corrected, unscaled: d/dt_a, d/dt_b
  double* fd_D;                  // [NB][9] FD diagonal (trans) block, unscaled
  double* fd_X;                  // [D][9] FD cross block J_a J_b^T, unscaled
  // linearization, two slots (s = LmState::cur: the current point; cur ^ 1: k_update_lin's candidate)
  double* J[2];
  double* V[2];
  double* g[2];
  int32_t spec;                  // speculative linearization: k_update_lin linearizes at every candidate
  double* scale_p;
  double* diag_p;
  double* Vinv;
  double* tp;
  double* scale_c;               // [n]
  double* diag_c;                // [n]
  double* camdiag;               // [n] diag(J^T J) camera columns, unscaled (obs + FD)
  double* camg;                  // [n] camera gradient, unscaled (obs + FD)
  // chunks and partials
  const int32_t* cam_loff;       // [NB+1] CSR: per camera block, offsets of its partials in cam_slab
  const int32_t* cam_lidx;
  const int32_t* s_loff;         // [nstile]: per band tile of S, the count of its partial tiles in S_slab, whose
                                 // offsets are s_lidx[s_lstride * tile ...] (rows padded to s_lstride, a multiple of 256)
  const int32_t* s_lidx;
  const int32_t* stile;          // [nstile] band tiles (R << 16) | C, R <= C, of the frame columns
  int32_t nstile;
  const int32_t* r_loff;         // [NB]: per block, the count of its rhs partials in S_slab (offsets: r_lidx rows of
                                 // r_lstride, a multiple of 256)
  const int32_t* r_lidx;
  int32_t s_lstride, r_lstride;  // padded row lengths of s_lidx / r_lidx (k_S_reduce reads a row's first 256
                                 // entries with no bound: its list loads go out beside the counts')
  double* cam_slab[2];
  double* S_slab;
  double* chunk_scal;            // [npu][kNScal] k_point_update scalars (per work unit)
  double* cam_wide[2];           // [NB][27] (wide chunks, global atomics)
  double* S_wide;                // [n][n]   (wide chunks, global atomics)
  double* zpre;                  // [257] Z_0 = U_00^-T of S's first diagonal tile, factored by k_S_reduce (+ failure)
  // exchange buffers (all-reduced across landmark shards)
  double* xchg_cam;              // [NB*27 + kXNum + nranks]: camera blocks, scalars, per-rank max |g| slots
                                 // (summed over the shards by the camera-block all-reduce)
  double* xcam_loc;              // the same, this rank's own (never all-reduced)
  double* xchg_cand;             // the same for the candidate (speculative chain: k_cam_reduce mode 1), local
  double* xtail;                 // merged exchange tail after the packed band of S (k_cam_finalize modes 1, 2):
                                 // camera gradient [6 NB] | diagonal [6 NB] | scalars [kXNum] | max |g| [nranks]
                                 // | FrameDistance cost
  int32_t rank, nranks;          // landmark shard of this solver
  double* S;                     // [n][n] reduced system (upper blocks), then its factor
  double* rhs;                   // [n]
  double* xchg_upd;              // [kUNum]
  double* xchg_chol;             // [kCNum]
  double* xc;                    // [n] camera solution (scaled)
  double* work;                  // [n] solver scratch
  const int32_t* fd_pair;        // [NB][NB] (I<J): 2 * FrameDistance residual coupling blocks I and J + (its frame a is block J), or -1
  int32_t assemble;              // this rank adds blockdiag(U) + FD + damping to S (rank 0 of a shard group)
  const int32_t* obs_pnt;        // [M] point (device order) of each observation
  const int32_t* obs_meta;       // [M] packed block / camera / freedom flags (kMeta*)
  const LinChunk* lchunks;       // [nlin] k_linearize workgroups
  const LinRound* lrounds;
  int32_t nlin;
  double* lin_scal[2];           // [nlin][kNScal] k_linearize scalars (cost, failures, |x|^2, max |g|)
  const int32_t* pu_units;       // [npu] k_point_update work units: round index, or -(chunk + 1) (wide chunk)
  int32_t npu;
  const struct SchurSeg* segs;   // [nseg] Schur work units
  int32_t nseg;
  const struct SchurBatch* sbatch;
  const int2* pinfo;             // [P] first cell, (first block << 8) | span (0: no Schur terms)
  const int4* cells;             // [ncell] first observation (-1: none), point, (block << 16) | number of
                                 // further observations, their offset in cell_obs
  const int4* pmx;               // [P] operand offset in the batch buffer, last window tile (-1: none),
                                 // observation of the first block (-1: use the cell records), first cell
  const int32_t* cell_obs;       // second and later observations of a cell
  const struct WideSeg* wsegs;   // [nwide] points wider than a segment window
  int32_t nwide;
  double* seg_fail;              // [nseg + nwide] point blocks whose damped inverse failed
  const int2* pairs;             // wide points: {(s << 16) | t local observation indices, (b_s << 16) | b_t}
  unsigned long long* stamps;    // diagnostic builds only: per-phase cycle counters (nullptr otherwise)
  // free intrinsics (SolveAllFrames(..., solve_cameras = true), slam.cpp:447-480): 7 columns per camera after
  // the 6 NB frame columns of S (nk = 0 when the intrinsics are constant)
  int32_t nk, kc0, ncam;         // nk = 7 ncam, kc0 = 6 NB
  double* Jk;                    // [M][14] corrected, unscaled d(uv)/dk of each observation
  double* KU;                    // [n][nk] intrinsics columns of J^T J, unscaled (frame rows, then the k block)
  double* kst;                   // [ncam][56] CameraStabilization corrected residual (7) and Jacobian (7x7)
  double* Yk;                    // [P][ncam][28] W_kp V~p^-1 of each free point (k_intr_schur -> k_intr_fk)
  double* kpart;                 // [(NB + 1) nsl][ncam][42] per-(block, slice) J_k^T J_k / J_k^T r / diagonal partials
  const int32_t* intr_boff;      // [NB + 2] per frame block (then the fixed frames' block NB): observations
  const int32_t* intr_bidx;      //   of non-fixed observations, in observation order
  double stab_b, stab_inv_b;     // CauchyLoss(stab_range): b = stab_range^2
};
constexpr int kMaxIntrCams = 4;  // cameras whose intrinsics the device solver can free at once

}  // namespace sg

#endif  // SG_BA_KERNELS_H_
