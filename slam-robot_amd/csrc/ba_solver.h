// ba_solver.h — host driver of the MI355X bundle-adjustment solver (one per sg_ba handle).
#ifndef SG_BA_SOLVER_H_
#define SG_BA_SOLVER_H_

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "ba_kernels.h"
#include "common.h"
#include "dbuf.h"
#include "hostio.h"
#include "hostmirror.h"

namespace sg {

void ValidateProblem(const sg_problem* p);

class Comm;  // RCCL communicator (comm.cpp)

class BaSolver {
 public:
  explicit BaSolver(const sg_device_options& dev);
  ~BaSolver();

  void Load(const sg_problem& p);
  // Pre-size every buffer that scales with the problem for up to F frames, P points and M observations (a
  // map's high-water mark), so that a later Load does not reallocate on its critical path.  Reallocating
  // drops the loaded structure (the next Load is a full one).
  void Reserve(int F, int P, int M);
  void Begin(const sg_solver_options& o);
  void Iterate(int n);
  void Sweep(int n);
  void Sync();
  void Summary(sg_solver_summary* s);
  void Download(sg_problem* p);
  void Solve(const sg_solver_options& o, sg_problem* p, sg_solver_summary* s);
  void Evaluate(double* residuals, double* cost, int32_t* nfail);
  void SetTiming(bool on);
  int KernelTimes(char* names, int names_len, double* ms, int32_t* counts, int max);
  int KernelWork(double* bytes, double* flops, int max);
  void CommInit(const void* id128, int nranks, int rank);
  void CommInitLocal(std::shared_ptr<struct LocalGroup> g, int rank);   // in-process test group (comm.h)
  void CommInitHost(int nranks, int rank, int (*fn)(double*, long long, int, void*), void* user);   // comm.h
  static void UniqueId(void* id128);

  void Info(sg_ba_info* out) const;

  // ReprojectMap (slam.cpp:523-548) over a whole map; used by the Slam facade.
  double ReprojectMap(sg_map* m);

  hipStream_t stream() const { return stream_; }
  int nranks() const;

 private:
  sg_device_options dev_;
  hipStream_t stream_ = nullptr;
  HostMirror mb_;   // mapped mailbox: [0, 1 KB) the LM state read back, then the solution download
  void ReadState(LmState* h);   // LmState via mb_ (a kernel writes it: no copy engine), stream synchronised
  void WaitStream(hipStream_t s);   // spin-wait for the stream's work (see ba_solver.hip)
  hipEvent_t ev_wait_ = nullptr;
  void EnqueueIterations(int n);
  hipEvent_t dev_marks_[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};   // SG_HOST_TIMING: device times in Load
  hipEvent_t ev_idle_ = nullptr;                                            //   the stream last seen idle (MarkIdle)
  hipEvent_t ev_idle_prev_ = nullptr;                                       //   the previous call's, at a load
  std::chrono::steady_clock::time_point idle_host_;
  bool idle_valid_ = false;
  void MarkIdle(hipStream_t s);
  void DevMark(hipStream_t s, int i);
  bool need_seq_ = true;   // the next iteration is the first of a solve (it computes the camera scale)
  std::unique_ptr<Comm> comm_;
  bool loaded_ = false;
  bool began_ = false;
  bool chol_window_ = true;
  bool chol_tiles_ = false;    // tiled register-resident band Cholesky (k_chol_tiles)
  bool chol_border_ = false;   // free intrinsics: k_chol_tiles on the frame band, then k_chol_border
  int border_flags_ = 0;       // its LDS placements (bit 0 q_K tiles, bit 1 candidate operands)
  size_t border_lds_max_ = 0;  // its dynamic LDS limit
  size_t tile_lds_ = 0;        // its dynamic LDS
  DBuf<double> Wg_;            // its back-substitution tiles W_KJ = U_KK^-1 U_KJ (+ the bottom half's)
  int chol_nd_ = 0;            // dissected band: tile rows the second workgroup factors bottom-up (0: one WG)
  int chol_ns_ = 7;            // ... and the separator's tile rows (<= 7)
  DBuf<int32_t> tflag_;        // dissected band hand-off counters {bottom done, top done}
  bool chol_cand_lds_ = false;   // candidate-pass operands staged in the Cholesky's LDS (small problems)
  int s_lstride_ = 256, r_lstride_ = 256;   // k_S_reduce's padded list rows (Dev::s_lstride / r_lstride)
  // tests only: force the dissected Cholesky's separator wait to time out (k_chol_tiles flags bit 2)
  bool chol_force_tmo_ = getenv("SG_CHOL_FORCE_TIMEOUT") && atoi(getenv("SG_CHOL_FORCE_TIMEOUT")) != 0;
  // SG_CHOL_ZPRE=0: k_chol_tiles factors D_0 itself instead of starting from k_S_reduce's Z_0 (A/B, tests)
  bool chol_zpre_off_ = getenv("SG_CHOL_ZPRE") && atoi(getenv("SG_CHOL_ZPRE")) == 0;
  bool pack_force_ = getenv("SG_PACK_S") != nullptr;   // pack/unpack S on one rank too (tests the path)
  // speculative linearization (k_update_lin: the candidate pass linearizes at the candidate; k_linearize runs
  // only in a solve's first iteration); SG_SPEC=0: k_point_update + k_linearize every iteration
  bool spec_ = !(getenv("SG_SPEC") && atoi(getenv("SG_SPEC")) == 0);
  size_t jslot_ = 0, cslot_ = 0;   // doubles per slot of J and cam_slab
  // merged exchange of landmark shards (ba_solver.hip, EnqueueIterations): 1 default (shards), 0 off (SG_XCHG_MERGE=0),
  // 2 forced on one rank too (SG_XCHG_MERGE=force, tests)
  int merge_ = getenv("SG_XCHG_MERGE") ? (std::string(getenv("SG_XCHG_MERGE")) == "force" ? 2 : atoi(getenv("SG_XCHG_MERGE")) != 0)
                                       : 1;
  size_t ntail_ = 0;   // doubles of the merged exchange's tail
  bool pending_decision_ = false;   // speculative chain: the last enqueued step awaits its decision
  int32_t nallreduce_ = 0;   // landmark-shard all-reduces issued (sg_ba_info.num_allreduces)
  // tests: issue the communicator's collectives on one rank too (SG_COMM_FORCE=1: RCCL with one rank is a copy)
  bool comm_force_ = getenv("SG_COMM_FORCE") && atoi(getenv("SG_COMM_FORCE")) == 1;
  size_t npack_ = 0;                                      // band of S + rhs, doubles (all-reduce size)
  bool stamp_on_ = false;
  int ncu_ = 256;                       // compute units (Schur segment count), queried once
  size_t tile_lds_set_ = 0;             // dynamic LDS last granted to k_chol_tiles
  size_t gchol_lds_max_ = 0;            // dynamic LDS granted to k_cholesky_global
  bool chol_gstage_ = false;            // k_cholesky_global stages panel rows in LDS
  std::unique_ptr<class Stager> stager_;   // batched structure uploads (stager.h)
  DBuf<unsigned long long> stamps_;

 public:
  // diagnostic: per-phase cycle counters of the stamped kernels (SG_STAMP=1)
  std::vector<unsigned long long> Stamps();

 private:
  // host copies of the structure
  int F_ = 0, P_ = 0, M_ = 0, NB_ = 0, n_ = 0, D_ = 0, ncam_ = 0;
  std::vector<int32_t> point_perm_;   // device order -> problem point
  std::vector<int32_t> obs_perm_;     // device order -> problem observation
  int band_tiles_ = 0;     // widest Cholesky envelope row (16-wide tiles)
  size_t npairs_ = 0;      // Schur observation pairs
  // Incremental problem update (replacing the per-call rebuild of slam.cpp:257-414):
  // the structure of the last Load.  A Load with the same structure (frames, cameras, freedom flags,
  // observation -> frame / point incidence, FrameDistance pairs) keeps the point order, the CSR, the sweep
  // chunks, Schur segments, pair and reduction lists and the Cholesky envelope, and uploads the values only.
  struct StructKey {
    int32_t ncam = -1, cams_free = 0, F = -1, P = -1, M = -1, D = -1;
    std::vector<int32_t> frame_camera, obs_frame, obs_point, dist_frame, dist_prev;
    std::vector<uint8_t> rot_free, trans_free, point_free;
  } skey_;
  int32_t full_loads_ = 0, value_loads_ = 0;
  bool SameStructure(const sg_problem& p) const;
  void SaveStructure(const sg_problem& p);
  void LoadValues(const sg_problem& p);
  void ResetState(hipStream_t s);

 public:
  // loads that rebuilt the structure / loads that re-uploaded values only
  void LoadCounts(int32_t* full, int32_t* values) const {
    *full = full_loads_;
    *values = value_loads_;
  }

 private:
  // device buffers
  DBuf<LmState> st_;
  DBuf<double> k_, q_, t_, X_, obs_pt_, J_, V_, g_, scale_p_, diag_p_, Vinv_, tp_, scale_c_, diag_c_, camdiag_,
      camg_, cam_slab_, S_slab_, chunk_scal_, cam_wide_, S_wide_, xchg_cam_, S_, rhs_, xchg_upd_,
      xchg_chol_, work_, fd_r_, fd_J_, fd_D_, fd_X_, red_, zpre_;
  DBuf<int32_t> frame_cam_, frame_block_, poff_, obs_frame_, fd_a_, fd_b_, fd_boff_, fd_bidx_, cam_loff_,
      cam_lidx_, s_loff_, s_lidx_, r_loff_, r_lidx_, mobs_frame_, mobs_point_, mframe_cam_;
  DBuf<uint8_t> rot_free_, trans_free_, pfree_, obs_fixed_;
  DBuf<int32_t> work_i_;   // Cholesky panel envelopes (panel_jmax)
  DBuf<int32_t> fd_pair_;
  DBuf<int32_t> pu_units_;   // k_point_update work units
  DBuf<int32_t> pack_off_;   // per panel offset of its band rows in the packed all-reduce buffer
  DBuf<double> Spk_;         // packed band of S + rhs (landmark shards)
  DBuf<int32_t> obs_pnt_, pairs_;   // Schur work lists
  DBuf<int32_t> obs_meta_;         // packed per-observation facts (kMeta*)
  DBuf<double> Jk_, KU_, kst_;     // free intrinsics (nk_ > 0)
  DBuf<double> Yk_, kpart_;        //   W_kp V~p^-1 per point and camera; per-block camera sums
  DBuf<int32_t> intr_boff_, intr_bidx_;   //   per-block observation lists
  int intr_nsl_ = 1;                      //   k_intr_fk workgroups per block list
  int nk_ = 0;                     // 7 * cameras when the intrinsics are free
  double stab_b_ = 25.0;
  DBuf<SchurSeg> segs_;
  DBuf<LinChunk> lchunks_d_;
  DBuf<LinRound> lrounds_d_;
  DBuf<double> lin_scal_;
  int nlin_ = 0;
  int lin_waves_ = 1;   // waves per k_linearize / k_update_lin chunk (2 when 2 nlin_ waves fit the chip at once)
  void LaunchLinearize(const Dev& d);
  void LaunchUpdateLin(const Dev& d);
  int npu_ = 0;
  DBuf<double> seg_fail_;
  int nseg_ = 0, nwide_ = 0, nstile_ = 0;
  double schur_mfma_ = 0.0;   // v_mfma_f64_16x16x4f64 tile updates per k_schur launch (KernelWork)
  double schur_rhs_ = 0.0;    // v_mfma_f64_4x4x4_4b_f64 rhs updates per k_schur launch
  double schur_useful_ = 0.0; // flops of the slots that multiply each point's own tiles (no zero tiles)
  DBuf<SchurBatch> sbatch_;
  DBuf<WideSeg> wsegs_;
  DBuf<int32_t> pinfo_, pmx_, cells_, cell_obs_, stile_;
  DBuf<double> rdg_;       // 1/U_jj of the factor
  DBuf<double> mk_, mq_, mt_, mX_, mobs_pt_, mobs_err_, mred_;
  HostIo io_;   // ReprojectMap's uploads and downloads (hostio.h)
  double range_b_ = 4.0, fd_target_ = 150.0, fd_b2_ = 225.0;
  // timing
  bool timing_ = false;
  struct KTimer {
    std::string name;
    std::vector<hipEvent_t> ev;  // pairs
    double total_ms = 0.0;
    int count = 0;
  };
  std::vector<KTimer> timers_;
  void TimedLaunchBegin(int id);
  void LaunchCholTiles(bool stamp, dim3 grid, const Dev& d, int flags);
  void TimedLaunchEnd(int id);
  void TimedLaunchBegin(int id, hipStream_t s);
  void TimedLaunchEnd(int id, hipStream_t s);
  void CollectTimes();
  Dev MakeDev();
  void AllReduceSum(double* buf, size_t n);
};

}  // namespace sg

#endif  // SG_BA_SOLVER_H_
