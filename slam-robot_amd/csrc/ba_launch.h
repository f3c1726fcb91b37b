// ba_launch.h — launch geometry and host launchers of the bundle-adjustment kernel families.
//
// The kernels live in one translation unit per family, each compiled for gfx950 on its own:
//   ba_sweep.hip  the Jacobian sweep and LM-step kernels: k_linearize, k_update_lin (speculative
//                 linearization), k_point_update, k_cam_reduce, k_upd_reduce, k_decide, k_evaluate,
//                 k_reproject_map
//   ba_schur.hip  the point elimination and reduced-system assembly: k_schur (+ the finalize workgroup),
//                 k_schur_wide, k_S_reduce, k_S_pack, k_cam_finalize
//   ba_chol.hip   the reduced-camera solves: k_chol_tiles (dissected band), k_chol_border (free intrinsics),
//                 k_cholesky_window, k_cholesky_global
//   ba_intr.hip   the free-intrinsics columns of SolveAllFrames(..., true): k_intr_*
// and the host driver (ba_solver.hip) reaches them only through the launchers below (plain host functions: no
// kernel symbol crosses a translation unit).
#ifndef SG_BA_LAUNCH_H_
#define SG_BA_LAUNCH_H_

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "ba_kernels.h"

namespace sg {

// ---- launch geometry the host driver shares with the kernels
constexpr int kRedThreads = 1024;      // k_cam_reduce / k_upd_reduce workgroup (>= kCamSlices * kCamV)
constexpr int kCholWS = 128;           // k_cholesky_window: LDS window columns
constexpr int kCholLd = kCholWS + 1;
constexpr size_t kCholLds = (size_t)kCholWS * kCholLd * sizeof(double);
constexpr int kJendSh = 512;           // panel band ends cached in LDS (n <= 8192)
constexpr int kCandMax = 1024;         // frames / FrameDistance residuals staged in LDS for the candidate pass
constexpr int kTB = 8;                 // k_chol_tiles: band width in tiles = waves
constexpr int kTileThreads = kTB * 64;
constexpr int kTileMaxNT = 400;        // k_chol_tiles: tile rows (dynamic LDS: x, z' 16 NT doubles each + band ends)
constexpr int kSplitMinNT = 13;        // dissected band from this many tile rows
constexpr int kBordThreads = 256;      // k_chol_border
constexpr int kIntrFkThreads = 256;    // k_intr_fk (the slices per block list stay ~256 observations)
constexpr int kIntrFinThreads = 256;   // k_intr_fin
// SG_STAMP=1 diagnostic stamp layout: [0, 64) per-wave phase sums, then the tiled Cholesky's per-phase trace,
// then k_update_lin's stamps
constexpr int kTraceK = 128;
constexpr int kUlStamp = 64 + 2 * kTraceK * 16;
// k_schur per-segment stamps (SG_STAMP=1): 8 words per segment from kSegStamp (tools/schur_seg_stamps.py)
constexpr int kSegStamp = kUlStamp + 16;
constexpr int kSegStampMax = 1024;

// ---- ba_sweep.hip
void LaunchLinearizeK(int waves, int grid, hipStream_t s, const Dev& d);
void LaunchUpdateLinK(bool stamp, int waves, int grid, hipStream_t s, const Dev& d);
void LaunchPointUpdateK(int grid, hipStream_t s, const Dev& d);
void LaunchCamReduceK(int grid, hipStream_t s, const Dev& d, int mode);
void LaunchUpdReduceK(hipStream_t s, const Dev& d, int fuse);
void LaunchDecideK(hipStream_t s, const Dev& d, int take);
void LaunchEvaluateK(int M, hipStream_t s, const Dev& d, double* resid, double* cost, int32_t* nfail);
void LaunchReprojectMapK(int M, int nb, hipStream_t s, const double* k, const double* q, const double* t,
                         const int32_t* frame_cam, const double* X, const double* obs_pt, const int32_t* obs_frame,
                         const int32_t* obs_point, double* err, double* partial);

// ---- ba_schur.hip
void LaunchCamFinalizeK(hipStream_t s, const Dev& d, int mode, int decide);
// fin: 0 none; 1 one workgroup runs k_cam_finalize's pass (one rank, mode 0); 2 its mode 1 (merged shards)
void LaunchSchurK(int nseg, int nwide, int fin, hipStream_t s, const Dev& d);
void LaunchSReduceK(int grid, hipStream_t s, const Dev& d, int amode, int pre = 0);
void LaunchSPackK(dim3 grid, hipStream_t s, double* S, int n, const int32_t* panel_jend, const int32_t* off,
                  int npanel, double* Spk, int dir);
// the merged chain's unpack + k_cam_finalize mode 2 (grid: LaunchSPackK's; one bookkeeping workgroup is added)
void LaunchSUnpackFinK(dim3 grid, hipStream_t s, const Dev& d, const int32_t* panel_jend, const int32_t* off,
                       int npanel, const double* Spk);

// ---- ba_intr.hip (free intrinsics): the linearization-side and Schur-side launches of one LM iteration
void LaunchIntrLinearizeK(hipStream_t s, const Dev& d, int n, int nk, int NB, int ncam, int M, int nsl);
void LaunchIntrSchurK(hipStream_t s, const Dev& d, int n, int nk, int NB, int ncam, int P, int nsl);
void LaunchIntrStepK(hipStream_t s, const Dev& d);

// ---- ba_chol.hip
// Grant every Cholesky kernel the dynamic LDS it may need, once per solver (a load never changes an attribute):
// returns the limits granted to k_chol_tiles, k_cholesky_global and k_chol_border.
void CholSetAttributes(size_t* tile_lds, size_t* gchol_lds, size_t* border_lds);
size_t border_lds_doubles(int NT, int flags, int F, int D, int n);   // k_chol_border's dynamic LDS (doubles)
size_t cand_lds_bytes(int F, int D, int n);   // the candidate pass's operands staged in a Cholesky's LDS
void LaunchCholTilesK(bool stamp, dim3 grid, size_t lds, hipStream_t s, const Dev& d, const int32_t* panel_jend,
                      double* Wg, int32_t* tflag, int nd, int flags);
void LaunchCholBorderK(int border_flags, size_t lds, hipStream_t s, const Dev& d, double* Wg);
void LaunchCholWindowK(bool stamp, hipStream_t s, const Dev& d, const int32_t* panel_jend, double* rdg);
void LaunchCholGlobalK(bool stage, size_t lds, hipStream_t s, const Dev& d, const int32_t* panel_jend, double* rdg);

}  // namespace sg

#endif  // SG_BA_LAUNCH_H_
