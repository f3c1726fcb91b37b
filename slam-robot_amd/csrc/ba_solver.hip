// ba_solver.hip — host driver of the MI355X-native Levenberg-Marquardt bundle adjustment (the reference's
// Slam::Run, slam.cpp:482-521, which hands the problem to Ceres 1.8 with SPARSE_SCHUR; restated on gfx950):
// problem load (work lists, the Schur segments, the Cholesky envelope, the structure-only incremental path), the
// per-iteration kernel chain and the host polls.  The kernels are in the family translation units listed in
// ba_launch.h; this file launches them through ba_launch.h's launchers and keeps only a few utility kernels
// (copies, buffer resets, the state hand-off, the solution download).
//
// One LM iteration = the kernel chain below, enqueued without host synchronisation; the accept/reject
// decision, trust-region update and termination tests run on the device, so a solve is a stream of identical
// iterations the host only polls for completion.  The default chain (one GPU, speculative linearization):
//   k_schur        (+ one workgroup: the camera finalize pass, FrameDistance / cost / gradient / LM diagonal)
//                  whitened point Jacobians, -E E^T into the segment's window tiles on the matrix cores
//   k_S_reduce     fixed-order reduce of the window tiles + blockdiag(U) + FrameDistance + damping -> S, rhs
//   k_chol_tiles   dissected tiled band Cholesky of S, back substitution, candidate poses
//   k_update_lin   point back substitution, model and candidate cost, and the linearization at the candidate
//   k_cam_reduce   the candidate's camera partials and update scalars reduced, and the LM decision (mode 2)
// Landmark shards add the exchanges of DESIGN.md 5 (pack, all-reduce, unpack) and the separate decision.
#include <hip/hip_runtime.h>

#include <chrono>
#include <string>
#include <thread>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <numeric>

#include "ba_solver.h"
#include "ba_device.h"
#include "ba_launch.h"
#include "comm.h"
#include "stager.h"

namespace sg {

// Word copy (8-byte words, grid-stride) between device and mapped host memory.
__global__ __launch_bounds__(256) void k_copy_u64(const unsigned long long* __restrict__ src,
                                                  unsigned long long* __restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// ================================================================================================
// Host driver

enum KernelId { kKLin = 0, kKCamReduce, kKCamFinal, kKSchur, kKSReduce, kKChol, kKPointUpd, kKUpdRed, kKDecide,
                kKXchg, kKNum };
static const char* kKernelNames[kKNum] = {"linearize", "cam_reduce", "cam_finalize", "schur", "S_reduce",
                                          "cholesky", "point_update", "upd_reduce", "decide", "exchange"};

void BaSolver::LaunchCholTiles(bool stamp, dim3 grid, const Dev& d, int flags) {
  // bordered: the frame band ends follow the arrowhead's panel ends in work_i_
  const int32_t* pj = (const int32_t*)work_i_.ptr + (chol_border_ ? (n_ + kCholNb - 1) / kCholNb : 0);
  if (chol_border_) flags |= 8;
  LaunchCholTilesK(stamp, grid, tile_lds_, stream_, d, pj, Wg_.ptr, tflag_.ptr, chol_nd_, flags | (chol_ns_ << 8));
  if (chol_border_) {
    const int ntf = (6 * NB_ + kCholNb - 1) / kCholNb;
    LaunchCholBorderK(border_flags_, border_lds_doubles(ntf, border_flags_, F_, D_, n_) * sizeof(double), stream_, d,
                      Wg_.ptr);
  }
}

BaSolver::BaSolver(const sg_device_options& dev) : dev_(dev) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw Error(SG_ENODEV, "no HIP device available");
  SG_REQUIRE(dev.device >= 0 && dev.device < ndev, SG_ENODEV, "device ordinal out of range");
  SG_REQUIRE(dev.precision == 0, SG_EINVAL,
             "sg_device_options.precision: only 0 (fp64, the reference's arithmetic) is implemented");
  SG_HIP_CHECK(hipSetDevice(dev.device));
  SG_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev.device) == hipSuccess && prop.multiProcessorCount > 0)
      ncu_ = prop.multiProcessorCount;
  }
  stager_.reset(new Stager());
  CholSetAttributes(&tile_lds_set_, &gchol_lds_max_, &border_lds_max_);
  st_.Resize(1);
  timers_.resize(kKNum);
  for (int i = 0; i < kKNum; ++i) timers_[i].name = kKernelNames[i];
}

BaSolver::~BaSolver() {
  for (auto& t : timers_)
    for (auto e : t.ev) (void)hipEventDestroy(e);
  if (ev_wait_) (void)hipEventDestroy(ev_wait_);
  if (ev_idle_) (void)hipEventDestroy(ev_idle_);
  if (ev_idle_prev_) (void)hipEventDestroy(ev_idle_prev_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void BaSolver::UniqueId(void* id128) { RcclComm::UniqueId(id128); }

void BaSolver::CommInit(const void* id128, int nranks, int rank) {
  SG_REQUIRE(!loaded_, SG_EINVAL, "sg_ba_comm_init must precede sg_ba_load (exchange buffers are sized by it)");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  comm_.reset(new RcclComm(id128, nranks, rank));
  dev_.nranks = nranks;
  dev_.rank = rank;
}

void BaSolver::CommInitLocal(std::shared_ptr<LocalGroup> g, int rank) {
  SG_REQUIRE(!loaded_, SG_EINVAL, "sg_ba_comm_init_local must precede sg_ba_load");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  comm_.reset(new LocalComm(std::move(g), rank));
  dev_.nranks = comm_->nranks();
  dev_.rank = rank;
}

void BaSolver::CommInitHost(int nranks, int rank, int (*fn)(double*, long long, int, void*), void* user) {
  SG_REQUIRE(!loaded_, SG_EINVAL, "sg_ba_comm_init_host must precede sg_ba_load");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  comm_.reset(new HostComm(nranks, rank, fn, user));
  dev_.nranks = comm_->nranks();
  dev_.rank = rank;
}

int BaSolver::nranks() const { return comm_ ? comm_->nranks() : 1; }

void BaSolver::AllReduceSum(double* buf, size_t n) {
  if (comm_ && (comm_->nranks() > 1 || comm_force_)) {
    comm_->AllReduceSum(buf, n, stream_);
    ++nallreduce_;
  }
}

__global__ __launch_bounds__(256) void k_fill_obs_pnt(const int32_t* __restrict__ poff, int32_t* __restrict__ obs_pnt,
                                                      int P) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  for (int o = poff[i]; o < poff[i + 1]; ++o) obs_pnt[o] = i;
}

void BaSolver::Load(const sg_problem& p) {
  static const bool host_timing = getenv("SG_HOST_TIMING") != nullptr;   // development aid: phase times
  auto lt0 = std::chrono::steady_clock::now();
  std::string lap_log;
  auto lap = [&](const char* what) {
    if (!host_timing) return;
    const auto t = std::chrono::steady_clock::now();
    char buf[96];
    snprintf(buf, sizeof(buf), " %s %.2f", what, std::chrono::duration<double, std::milli>(t - lt0).count());
    lap_log += buf;
    lt0 = t;
  };
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  // a device mark at the load's start, with its host time: the GPU time from here to the last mark against the
  // host's wall time tells a late device (its queue started late) from a late host (the waiting thread)
  auto load_t0 = std::chrono::steady_clock::now();
  const bool idle_valid_prev = idle_valid_;
  const double idle_gap_host =
      idle_valid_ ? std::chrono::duration<double, std::milli>(load_t0 - idle_host_).count() : 0.0;
  std::swap(ev_idle_, ev_idle_prev_);   // (this load's own waits re-mark ev_idle_)
  if (host_timing) DevMark(stream_, 4);
  {
    // Everything that can reject this rank's problem runs before the first collective, and the verdict rides
    // in that collective (2: some rank's problem is invalid), so that all ranks fail together instead of
    // leaving the others blocked in an all-reduce.
    int vcode = SG_OK;
    std::string verr;
    try {
      ValidateProblem(&p);
      SG_REQUIRE(!p.cameras_free || (p.num_cameras <= kMaxIntrCams && nranks() == 1), SG_EINVAL,
                 "free intrinsics: at most 4 cameras, on one rank (landmark shards keep the intrinsics constant)");
      SG_REQUIRE(p.num_cameras <= 0xff, SG_EINVAL, "too many cameras for the device solver");
      int nfree = 0;
      for (int f = 0; f < p.num_frames; ++f) nfree += (p.frame_rot_free[f] || p.frame_trans_free[f]) ? 1 : 0;
      SG_REQUIRE(nfree < 0xffff, SG_EINVAL, "too many free frames for the device solver");
      std::vector<int32_t> cnt(p.num_points, 0);
      for (int o = 0; o < p.num_obs; ++o)
        SG_REQUIRE(++cnt[p.obs_point[o]] < 65536, SG_EINVAL, "a point has 65536 or more observations");
    } catch (const Error& e) {
      vcode = e.code;
      verr = e.what();
    }
    // incremental update: every rank must take the same path (the full path has a load-time all-reduce)
    double changed = vcode != SG_OK ? 2.0 : (loaded_ && SameStructure(p)) ? 0.0 : 1.0;
    if (comm_ && (comm_->nranks() > 1 || comm_force_)) {
      DBuf<double> flag;
      flag.Upload(std::vector<double>{changed}, stream_);
      comm_->AllReduceMax(flag.ptr, 1, stream_);
      SG_HIP_CHECK(hipMemcpyAsync(&changed, flag.ptr, sizeof(double), hipMemcpyDeviceToHost, stream_));
      SG_HIP_CHECK(hipStreamSynchronize(stream_));
    }
    if (vcode != SG_OK) throw Error(vcode, verr);
    if (changed == 2.0) throw Error(SG_EINVAL, "another landmark shard's problem failed validation");
    if (changed == 0.0) {
      LoadValues(p);
      lap("values");
      if (host_timing) fprintf(stderr, "[sg] Load phases (ms):%s\n", lap_log.c_str());
      return;
    }
  }
  // Full path: the structure and every device list are rebuilt below.  Until that completes, this solver
  // holds no usable problem: a failure part way (a device allocation, a hipFuncSetAttribute) must not leave
  // the previous problem's structure key matching a later load's value-only path.
  loaded_ = false;
  began_ = false;
  skey_ = StructKey{};
  stager_->Clear();
  F_ = p.num_frames;
  P_ = p.num_points;
  M_ = p.num_obs;
  D_ = p.num_dist;
  ncam_ = p.num_cameras;
  range_b_ = p.range * p.range;
  fd_target_ = p.dist_target;
  fd_b2_ = p.dist_range * p.dist_range;
  // camera blocks: every frame with a free rotation or translation
  std::vector<int32_t> frame_block(F_, -1);
  NB_ = 0;
  for (int f = 0; f < F_; ++f)
    if (p.frame_rot_free[f] || p.frame_trans_free[f]) frame_block[f] = NB_++;
  nk_ = p.cameras_free ? 7 * ncam_ : 0;
  n_ = 6 * NB_ + nk_;   // frame columns, then the free intrinsics
  stab_b_ = p.stab_range * p.stab_range;
  lap("blocks");
  // point order: by first free block (points without free-frame observations last)
  std::vector<int32_t> pfirst(P_, NB_), plast(P_, -1), pcount(P_, 0);
  for (int o = 0; o < M_; ++o) {
    const int pt = p.obs_point[o], b = frame_block[p.obs_frame[o]];
    pcount[pt]++;
    if (b >= 0) {
      pfirst[pt] = std::min(pfirst[pt], b);
      plast[pt] = std::max(plast[pt], b);
    }
  }
  // stable counting sort on the key pfirst in [0, NB]
  point_perm_.resize(P_);
  std::vector<int32_t> inv_perm(P_);
  {
    std::vector<int32_t> bstart(NB_ + 2, 0);
    for (int i = 0; i < P_; ++i) bstart[pfirst[i] + 1]++;
    for (int b = 0; b <= NB_; ++b) bstart[b + 1] += bstart[b];
    for (int i = 0; i < P_; ++i) {
      const int pos = bstart[pfirst[i]]++;
      point_perm_[pos] = i;
      inv_perm[i] = pos;
    }
  }
  // the first / last free block of each point in device order (the work-list builders below read them per point)
  std::vector<int32_t> dfirst(P_), dlast(P_);
  for (int i = 0; i < P_; ++i) {
    dfirst[i] = pfirst[point_perm_[i]];
    dlast[i] = plast[point_perm_[i]];
  }
  lap("point-order");
  // observations: CSR by device point order (stable in problem order)
  std::vector<int32_t> poff(P_ + 1, 0);
  for (int o = 0; o < M_; ++o) poff[inv_perm[p.obs_point[o]] + 1]++;
  for (int i = 0; i < P_; ++i) poff[i + 1] += poff[i];
  obs_perm_.assign(M_, 0);
  {
    std::vector<int32_t> fill(poff.begin(), poff.end() - 1);
    for (int o = 0; o < M_; ++o) obs_perm_[fill[inv_perm[p.obs_point[o]]]++] = o;
    // within a point: observations of constant frames first, then by camera block (stable), so that a point
    // observed once in every block of its span finds the observation of block b at a fixed offset (k_schur)
    // (a stable insertion sort: a point has a handful of observations, and std::stable_sort allocates a
    // buffer per call)
    for (int i = 0; i < P_; ++i) {
        int32_t* v = obs_perm_.data() + poff[i];
        const int k = poff[i + 1] - poff[i];
        if (k > 64) {
          std::stable_sort(v, v + k, [&](int a, int b) {
            return frame_block[p.obs_frame[a]] < frame_block[p.obs_frame[b]];
          });
          continue;
        }
        for (int x = 1; x < k; ++x) {
          const int32_t o = v[x];
          const int key = frame_block[p.obs_frame[o]];
          int y = x - 1;
          while (y >= 0 && frame_block[p.obs_frame[v[y]]] > key) {
            v[y + 1] = v[y];
            --y;
          }
          v[y + 1] = o;
        }
      }
  }
  std::vector<double> obs_pt(2 * (size_t)M_);
  std::vector<int32_t> obs_frame(M_);
  std::vector<uint8_t> obs_fixed(M_), pfree(P_);
  std::vector<double> X(4 * (size_t)P_);
  for (int i = 0; i < P_; ++i) {
    const int pt = point_perm_[i];
    pfree[i] = p.point_free[pt];
    for (int a = 0; a < 4; ++a) X[4 * i + a] = p.X[4 * pt + a];
  }
  std::vector<int32_t> obs_meta(M_);
  {
    // per frame: the frame part of the packed observation word
    std::vector<int32_t> fmeta(F_);
    for (int f = 0; f < F_; ++f)
      fmeta[f] = (frame_block[f] + 1) | (p.frame_camera[f] << kMetaCamShift) | (p.frame_rot_free[f] ? kMetaRot : 0) |
                 (p.frame_trans_free[f] ? kMetaTrans : 0);
    for (int o = 0; o < M_; ++o) {
      const int src = obs_perm_[o], f = p.obs_frame[src];
      const bool pf = p.point_free[p.obs_point[src]] != 0;
      obs_pt[2 * o] = p.obs_pt[2 * src];
      obs_pt[2 * o + 1] = p.obs_pt[2 * src + 1];
      obs_frame[o] = f;
      obs_fixed[o] = frame_block[f] < 0 && !pf && !p.cameras_free;
      obs_meta[o] = fmeta[f] | (pf ? kMetaPfree : 0) | (obs_fixed[o] ? kMetaFixed : 0);
    }
  }
  lap("obs-csr");
  // upload batch 1 — poses, intrinsics, points (current slot; the candidate slot is a device copy) and the
  // observation arrays: its pinned copy and DMA overlap the host's work-list construction below (stager.h)
  hipStream_t s = stream_;
  Stager& stg = *stager_;
  stg.ResetBytes();
  stg.AddInto(k_, std::max<size_t>(14 * (size_t)ncam_, 1),
              ncam_ > 0 ? std::vector<double>(p.k, p.k + 7 * ncam_) : std::vector<double>{0.0});
  stg.AddInto(q_, 8 * (size_t)F_, std::vector<double>(p.q, p.q + 4 * F_));
  stg.AddInto(t_, 6 * (size_t)F_, std::vector<double>(p.t, p.t + 3 * F_));
  stg.AddInto(X_, 8 * (size_t)P_, X);
  stg.Add(frame_cam_, std::vector<int32_t>(p.frame_camera, p.frame_camera + F_));
  stg.Add(frame_block_, frame_block);
  stg.Add(rot_free_, std::vector<uint8_t>(p.frame_rot_free, p.frame_rot_free + F_));
  stg.Add(trans_free_, std::vector<uint8_t>(p.frame_trans_free, p.frame_trans_free + F_));
  stg.Add(pfree_, pfree);
  stg.Add(poff_, poff);
  stg.Add(obs_pt_, obs_pt);
  stg.Add(obs_frame_, obs_frame);
  stg.Add(obs_fixed_, obs_fixed);
  stg.Add(obs_meta_, obs_meta.empty() ? std::vector<int32_t>{0} : obs_meta);
  if (host_timing) DevMark(s, 0);
  stg.Flush(s);
  {
    auto dup = [&](double* base, size_t half) {   // candidate slot = current slot
      if (half)   // a kernel, not a copy-engine hipMemcpyAsync (see hostmirror.h)
        hipLaunchKernelGGL(k_copy_u64, dim3((unsigned)std::min<size_t>(256, (half + 255) / 256)), dim3(256), 0, s,
                           reinterpret_cast<const unsigned long long*>(base),
                           reinterpret_cast<unsigned long long*>(base + half), half);
    };
    dup(k_.ptr, 7 * (size_t)ncam_);
    dup(q_.ptr, 4 * (size_t)F_);
    dup(t_.ptr, 3 * (size_t)F_);
    dup(X_.ptr, 4 * (size_t)P_);
    // the point of every observation (device order) from the CSR, on the device
    obs_pnt_.Resize(std::max(M_, 1));
    if (P_ > 0)
      hipLaunchKernelGGL(k_fill_obs_pnt, dim3((P_ + 255) / 256), dim3(256), 0, s, (const int32_t*)poff_.ptr,
                         obs_pnt_.ptr, P_);
    SG_HIP_CHECK(hipGetLastError());
  }
  lap("upload-1");
  // Schur work lists (see SchurSeg): the cells of every free point (one per block of its span, with the
  // point's observations in that block), segments of consecutive points whose columns fit kSchurTW tiles of
  // S, their batches, and each wide point's observation pairs (s <= t, both on free frames).
  std::vector<int32_t> pinfo(2 * (size_t)std::max(P_, 1), 0), pmx(4 * (size_t)std::max(P_, 1), 0), cells, cell_obs;
  std::vector<SchurSeg> segs;
  std::vector<SchurBatch> sbatch;
  std::vector<WideSeg> wsegs;
  std::vector<int32_t> pairs_flat;   // int2 per pair (wide points)
  int s_off = 0;
  // k_linearize decomposition (see LinChunk): rounds of whole points (<= kLinObs observations), up to
  // maxr rounds per chunk sharing one camera window; fewer rounds per chunk on small problems so that the
  // grid still fills the chip.
  std::vector<LinRound> lrounds;
  std::vector<LinChunk> lchunks;
  int lcam_off = 0;
  {
    int maxr = std::max(1, std::min(kLinMaxRounds, M_ / (kLinObs * 1024)));
    auto kobs = [&](int i) { return poff[i + 1] - poff[i]; };
    auto constonly = [&](int i) { return dfirst[i] >= NB_; };
    auto pspan = [&](int i) { return constonly(i) ? 0 : dlast[i] - dfirst[i] + 1; };
    for (int i = 0; i < P_;) {
      LinChunk c{};
      c.p0 = i;
      c.r0 = (int)lrounds.size();
      if (kobs(i) > kLinObs || pspan(i) > kLinNbMax) {
        c.wide = 1;
        for (int o = poff[i]; o < poff[i + 1]; o += kLinObs)
          lrounds.push_back(LinRound{o, std::min(o + kLinObs, poff[i + 1]), i, i + 1});
        c.p1 = ++i;
      } else {
        const bool co = constonly(i);
        int lo = co ? 0 : dfirst[i], hi = co ? -1 : dlast[i];
        int j = i, nr = 0;
        LinRound R{poff[i], poff[i], i, i};
        while (j < P_) {
          if (kobs(j) > kLinObs || pspan(j) > kLinNbMax || constonly(j) != co) break;
          int l2 = lo, h2 = hi;
          if (!co) {
            l2 = std::min(lo, dfirst[j]);
            h2 = std::max(hi, dlast[j]);
            if (h2 - l2 + 1 > kLinNbMax) break;
          }
          if (R.o1 - R.o0 + kobs(j) > kLinObs || R.p1 - R.p0 >= kLinPts) {
            if (nr + 1 >= maxr) break;
            lrounds.push_back(R);
            ++nr;
            R = LinRound{poff[j], poff[j], j, j};
          }
          R.o1 += kobs(j);
          R.p1 = j + 1;
          lo = l2;
          hi = h2;
          ++j;
        }
        lrounds.push_back(R);
        c.p1 = j;
        c.b_lo = lo;
        c.nb = co ? 0 : hi - lo + 1;
        i = j;
      }
      c.r1 = (int)lrounds.size();
      c.cam_off = lcam_off;
      lcam_off += c.nb * kCamV;
      lchunks.push_back(c);
    }
  }
  nlin_ = (int)lchunks.size();
  // two waves per chunk (its rounds split between them) while the doubled grid still fits the chip at three
  // waves per SIMD (k_linearize's occupancy): config 2's ~1.5 k chunks; one wave per chunk when there are more
  // chunks than that (config 5, the scaled sweep), where the second wave only adds the combine.  (A producer /
  // consumer split of a chunk's rounds over two waves was measured slower at config 5: DESIGN.md 8.)
  lin_waves_ = 2 * (long long)nlin_ <= 12LL * ncu_ ? 2 : 1;
  if (const char* e = getenv("SG_LIN_WAVES")) lin_waves_ = atoi(e) == 2 ? 2 : 1;   // A/B and tests
  std::vector<int32_t> pu_units;   // k_point_update work units: a round index, or -(chunk + 1) for wide chunks
  for (int c = 0; c < nlin_; ++c) {
    lchunks[c].u0 = (int)pu_units.size();   // k_update_lin writes the units' scalars
    if (lchunks[c].wide)
      pu_units.push_back(-(c + 1));
    else
      for (int r = lchunks[c].r0; r < lchunks[c].r1; ++r) pu_units.push_back(r);
  }
  npu_ = (int)pu_units.size();
  if (pu_units.empty()) pu_units.push_back(0);
  lap("lin-lists");
  std::vector<int32_t> obs_blk(M_);
  for (int o = 0; o < M_; ++o) obs_blk[o] = frame_block[obs_frame[o]];
  // span in blocks of a free point's Schur terms (0: none)
  std::vector<int32_t> ssp(std::max(P_, 1));
  for (int i = 0; i < P_; ++i) ssp[i] = (pfree[i] && dfirst[i] < NB_) ? dlast[i] - dfirst[i] + 1 : 0;
  auto sspan = [&](int i) { return ssp[i]; };
  std::vector<int32_t> simple_obs(std::max(P_, 1), -1);   // observation of the first block if one per block
  int ncell = 0;
  npairs_ = 0;
  schur_mfma_ = 0.0;
  schur_rhs_ = 0.0;
  schur_useful_ = 0.0;
  {
    std::vector<std::pair<int, int>> bo;
    cells.reserve(4 * (size_t)M_ + 4);
    cell_obs.reserve((size_t)M_ / 4 + 1);
    for (int i = 0; i < P_; ++i) {
      size_t kb = 0;
      for (int o = poff[i]; o < poff[i + 1]; ++o) kb += obs_blk[o] >= 0;
      if (pfree[i]) npairs_ += kb * (kb + 1) / 2;
      const int sp = sspan(i);
      if (sp == 0 || sp > kSegNbMax) continue;
      const int pf = dfirst[i];
      pinfo[2 * i] = (int)(cells.size() / 4);
      pinfo[2 * i + 1] = (pf << 8) | sp;
      bo.clear();
      for (int o = poff[i]; o < poff[i + 1]; ++o)
        if (obs_blk[o] >= 0) bo.emplace_back(obs_blk[o], o);
      if (!std::is_sorted(bo.begin(), bo.end())) std::sort(bo.begin(), bo.end());   // sorted at load already
      {
        bool one = (int)bo.size() == sp;   // observations sorted by block at load: consecutive
        for (int q = 0; one && q < sp; ++q) one = bo[q].first == pf + q && bo[q].second == bo[0].second + q;
        if (one) simple_obs[i] = bo[0].second;
      }
      size_t k = 0;
      for (int b = pf; b < pf + sp; ++b) {
        // {first observation or -1, point, (block << 16) | further observations, their offset in cell_obs}
        int o0 = -1;
        if (k < bo.size() && bo[k].first == b) o0 = bo[k++].second;
        const int k1 = (int)cell_obs.size();
        while (k < bo.size() && bo[k].first == b) cell_obs.push_back(bo[k++].second);
        cells.insert(cells.end(), {o0, i, (int)(((unsigned)b << 16) | (unsigned)(cell_obs.size() - k1)), k1});
      }
    }
    ncell = (int)cells.size() / 4;
    if (cells.empty()) cells.assign(4, 0);
    if (cell_obs.empty()) cell_obs.push_back(0);
  }
  {
    // Segments: one per CU (the workgroup's LDS holds one per CU; fewer, longer segments write fewer partial tiles
    // and keep the producer/consumer pipeline full: 256 / 384 / 512 / 768 / 1024 segments measured 35.9 / 46.5 /
    // 40.9 / 47.8 / 53.0 us at C2, profiles/r2 segs sweep), balanced by the work of the busiest MFMA wave rather
    // than by point count (round 5): a point costs its slots on that wave, ceil(schur_aug_base(jhi + 1) /
    // kSchurCWaves) with jhi its last tile in the segment's window, plus kSegPointCost for its fetch (the MFMA
    // waves are the bound once the producers are pipelined; 0 / 1 / 2 / 4 / 8 measured C5 k_schur 292 / 260 /
    // 245 / 238 / 244 us against 259 with equal point counts, profiles/r5_s1_schur_ab.log).  The cap starts at the
    // estimated total / CUs (each point's tiles counted from its own first tile) and is raised while the window
    // breaks push the count past the CUs: two passes at C2 and C5.
    constexpr int kSegMinPts = 16;      // small problems: no segment of a handful of points
    constexpr int kSegPointCost = 4;
    auto point_cost = [&](int j, int tile0) {
      const int sp = sspan(j);
      if (sp == 0) return kSegPointCost;
      const int e = (6 * (dfirst[j] + sp) - 1) / 16 - tile0;
      return kSegPointCost + (schur_aug_base(e + 1) + kSchurCWaves - 1) / kSchurCWaves;
    };
    std::vector<int32_t> seg_end;   // exclusive end of each planned segment, in point order
    auto plan = [&](long long cap) {
      seg_end.clear();
      for (int i = 0; i < P_;) {
        if (sspan(i) > kSegNbMax) {   // a wide point: k_schur_wide (the build loop below)
          ++i;
          continue;
        }
        int clo = INT32_MAX, chi = -1, j = i;
        long long acc = 0;
        while (j < P_) {
          const int sp = sspan(j);
          if (sp > kSegNbMax) break;
          int l2 = clo, h2 = chi;
          if (sp > 0) {
            const int pf = dfirst[j];
            l2 = std::min(clo, 6 * pf);
            h2 = std::max(chi, 6 * (pf + sp));
            if ((h2 + 15) / 16 - l2 / 16 > kSchurTW) break;
          }
          const int c = point_cost(j, l2 == INT32_MAX ? 0 : l2 / 16);
          if (j - i >= kSegMinPts && acc + c > cap) break;
          acc += c;
          clo = l2;
          chi = h2;
          ++j;
        }
        seg_end.push_back(j);
        i = j;
      }
    };
    {
      long long est = 0;
      for (int j = 0; j < P_; ++j)
        if (sspan(j) <= kSegNbMax) est += point_cost(j, sspan(j) ? 6 * dfirst[j] / 16 : 0);
      long long cap = std::max(1LL, (est + ncu_ - 1) / ncu_);
      for (int pass = 0; pass < 8; ++pass) {
        plan(cap);
        if ((int)seg_end.size() <= ncu_) break;
        cap += cap * (seg_end.size() - ncu_) * 3 / (2 * ncu_) + cap / 200 + 1;
      }
    }
    size_t next_seg = 0;
    int cnext = 0;
    for (int i = 0; i < P_;) {
      if (sspan(i) > kSegNbMax) {
        WideSeg w{};
        w.p = i;
        w.pair_lo = (int)pairs_flat.size() / 2;
        for (int os = poff[i]; os < poff[i + 1]; ++os) {
          if (obs_blk[os] < 0) continue;
          for (int ot = os; ot < poff[i + 1]; ++ot) {
            if (obs_blk[ot] < 0) continue;
            pairs_flat.push_back(((os - poff[i]) << 16) | (ot - poff[i]));
            pairs_flat.push_back((obs_blk[os] << 16) | obs_blk[ot]);
          }
        }
        w.pair_hi = (int)pairs_flat.size() / 2;
        wsegs.push_back(w);
        ++i;
        continue;
      }
      SchurSeg sg{};
      sg.p0 = i;
      int clo = INT32_MAX, chi = -1, blo = INT32_MAX, bhi = -1;   // columns [clo, chi), blocks [blo, bhi]
      int j = i;
      SG_REQUIRE(next_seg < seg_end.size() && seg_end[next_seg] > i, SG_EINVAL, "Schur segment plan out of step");
      const int jend = seg_end[next_seg++];
      while (j < jend) {
        const int sp = sspan(j);
        if (sp > kSegNbMax) break;
        if (sp > 0) {
          const int pf = dfirst[j];
          const int l2 = std::min(clo, 6 * pf), h2 = std::max(chi, 6 * (pf + sp));
          if ((h2 + 15) / 16 - l2 / 16 > kSchurTW) break;
          clo = l2;
          chi = h2;
          blo = std::min(blo, pf);
          bhi = std::max(bhi, pf + sp - 1);
        }
        ++j;
      }
      sg.p1 = j;
      if (chi >= 0) {
        sg.t0 = clo / 16;
        sg.ntw = (chi + 15) / 16 - sg.t0;
        sg.b_lo = blo;
        sg.nb = bhi - blo + 1;
      }
      // k_schur's asm chain (schur_chain.h) is entered at an offset computed from a point's last window tile:
      // every point must end inside the window (jhi <= kSchurTW - 1)
      SG_REQUIRE(sg.ntw <= kSchurTW, SG_EINVAL, "Schur segment window wider than kSchurTW");
      sg.s_off = s_off;
      s_off += sg.ntw * (sg.ntw + 1) / 2 * 256 + 16 * sg.ntw;
      // last window tile of each point's columns (-1: no Schur terms)
      auto pjhi = [&](int k) {
        const int sp = sspan(k);
        return sp == 0 ? -1 : (6 * (dfirst[k] + sp) - 1 - 16 * sg.t0) / 16;
      };
      sg.bt0 = (int)sbatch.size();
      for (int k = i; k < j;) {
        SchurBatch B{};
        B.p0 = k;
        B.c0 = cnext;
        int nc = 0, nx = 0;
        while (k < j && k - B.p0 < kSchurBatchPts && nx + 64 * (pjhi(k) + 1) <= kSchurXCap &&
               nc + sspan(k) <= 64 * kSchurCellWaves) {
          SG_REQUIRE(pjhi(k) < sg.ntw, SG_EINVAL, "point ends outside its Schur segment window");
          pmx[4 * k] = nx;
          pmx[4 * k + 1] = pjhi(k);
          pmx[4 * k + 2] = simple_obs[k];
          pmx[4 * k + 3] = nc;
          nx += 64 * (pjhi(k) + 1);
          schur_mfma_ += schur_aug_base(pjhi(k) + 1) - (pjhi(k) + 1);   // window tiles (16x16x4)
          schur_rhs_ += pjhi(k) + 1;                                      // rhs slots (4x4x4, 4 blocks)
          if (pjhi(k) >= 0) {   // the slots that multiply the point's own tiles (the rest multiply zeros)
            const double nu = pjhi(k) - (6 * dfirst[k] - 16 * sg.t0) / 16 + 1;
            schur_useful_ += 2048.0 * nu * (nu + 1) / 2 + 512.0 * nu;
          }
          nc += sspan(k++);
        }
        B.p1 = k;
        B.c1 = B.c0 + nc;
        cnext += nc;
        sbatch.push_back(B);
      }
      sg.bt1 = (int)sbatch.size();
      segs.push_back(sg);
      i = j;
    }
    SG_REQUIRE(cnext == ncell, SG_EINVAL, "Schur cells out of step with the batches");
  }
  nseg_ = (int)segs.size();
  nwide_ = (int)wsegs.size();
  if (pairs_flat.empty()) pairs_flat.assign(2, 0);
  lap("segments");
  // deterministic reduction lists: for every camera block, the slab offsets of the chunk partials that cover
  // it (fixed chunk order), and of the segments' rhs partials
  std::vector<int32_t> cam_loff(NB_ + 1, 0), cam_lidx, r_loff(NB_ + 1, 0), r_lidx;
  {
    std::vector<std::vector<int32_t>> cl(NB_), rl(NB_);
    for (const LinChunk& ch : lchunks) {
      if (ch.wide || ch.nb == 0) continue;
      for (int i = 0; i < ch.nb; ++i) cl[ch.b_lo + i].push_back(ch.cam_off + i * kCamV);
    }
    for (const SchurSeg& sg : segs) {   // rhs partial of block I: window columns 6 I - 16 t0 ..
      const int ntile = sg.ntw * (sg.ntw + 1) / 2;
      for (int i = 0; i < sg.nb; ++i)
        rl[sg.b_lo + i].push_back(sg.s_off + 256 * ntile + 6 * (sg.b_lo + i) - 16 * sg.t0);
    }
    size_t rmax = 0;
    for (int b = 0; b < NB_; ++b) rmax = std::max(rmax, rl[b].size());
    r_lstride_ = (int)std::max<size_t>(256, (rmax + 255) / 256 * 256);   // rows padded (k_S_reduce's unbounded reads)
    r_lidx.assign((size_t)std::max(NB_, 1) * r_lstride_, 0);
    for (int b = 0; b < NB_; ++b) {
      cam_loff[b + 1] = cam_loff[b] + (int)cl[b].size();
      cam_lidx.insert(cam_lidx.end(), cl[b].begin(), cl[b].end());
      r_loff[b] = (int)rl[b].size();
      std::copy(rl[b].begin(), rl[b].end(), r_lidx.begin() + (size_t)b * r_lstride_);
    }
    if (cam_lidx.empty()) cam_lidx.push_back(0);
  }
  lap("reduce-lists");
  // FrameDistance
  std::vector<int32_t> fd_a(p.dist_frame, p.dist_frame + D_), fd_b(p.dist_prev, p.dist_prev + D_);
  std::vector<int32_t> fd_boff(NB_ + 1, 0), fd_bidx;
  {
    std::vector<std::vector<int32_t>> lists(NB_);
    for (int dd = 0; dd < D_; ++dd) {
      const int ba = frame_block[fd_a[dd]], bb = frame_block[fd_b[dd]];
      if (ba >= 0) lists[ba].push_back(2 * dd);
      if (bb >= 0) lists[bb].push_back(2 * dd + 1);
    }
    for (int b = 0; b < NB_; ++b) {
      fd_boff[b + 1] = fd_boff[b] + (int)lists[b].size();
      fd_bidx.insert(fd_bidx.end(), lists[b].begin(), lists[b].end());
    }
  }
  lap("fd");
  // Cholesky panel envelopes: block column J's first nonzero block row lo(J)
  std::vector<int32_t> lo_blk(NB_);
  for (int b = 0; b < NB_; ++b) lo_blk[b] = b;
  {
    // exact envelope from the observations of each free point (pairs of blocks it couples)
    for (int i = 0; i < P_; ++i) {
      const int pt = point_perm_[i];
      if (pfirst[pt] >= NB_) continue;
      if (!p.point_free[pt]) continue;
      const int lo = pfirst[pt];
      for (int o = poff[i]; o < poff[i + 1]; ++o) {
        const int b = frame_block[obs_frame[o]];
        if (b >= 0) lo_blk[b] = std::min(lo_blk[b], lo);
      }
    }
    for (int dd = 0; dd < D_; ++dd) {
      const int ba = frame_block[fd_a[dd]], bb = frame_block[fd_b[dd]];
      if (ba >= 0 && bb >= 0) {
        const int hi3 = std::max(ba, bb), lo3 = std::min(ba, bb);
        lo_blk[hi3] = std::min(lo_blk[hi3], lo3);
      }
    }
  }
  // Landmark shards: S is summed over every rank's points, so each rank must factor it with the envelope of
  // the whole problem (the union of the shards' envelopes), not of its own points.  One max all-reduce of
  // -lo(J) at load time.
  if (comm_ && (comm_->nranks() > 1 || comm_force_) && NB_ > 0) {
    std::vector<double> neg(NB_);
    for (int b = 0; b < NB_; ++b) neg[b] = -(double)lo_blk[b];
    DBuf<double> env;
    env.Upload(neg, stream_);
    comm_->AllReduceMax(env.ptr, (size_t)NB_, stream_);
    SG_HIP_CHECK(hipMemcpyAsync(neg.data(), env.ptr, NB_ * sizeof(double), hipMemcpyDeviceToHost, stream_));
    SG_HIP_CHECK(hipStreamSynchronize(stream_));
    for (int b = 0; b < NB_; ++b) lo_blk[b] = (int)(-neg[b]);
  }
  const int npanel = (n_ + kCholNb - 1) / kCholNb;
  std::vector<int32_t> panel_jmax(std::max(npanel, 1), 0), panel_bend(std::max(npanel, 1), 0);
  for (int pk = 0; pk < npanel; ++pk) {
    const int row_hi = std::min(n_, (pk + 1) * kCholNb) - 1;   // last row of the panel
    const int blk_hi = row_hi / 6;
    int jmax = (pk + 1) * kCholNb;
    // columns j whose envelope starts at or before the panel's last row block
    for (int b = 0; b < NB_; ++b)
      if (lo_blk[b] <= blk_hi) jmax = std::max(jmax, 6 * b + 6);
    jmax = std::min(jmax, n_);
    panel_jmax[pk] = std::min(n_, (jmax + kCholNb - 1) / kCholNb * kCholNb);   // band end, 16-aligned
    if (nk_) {   // the intrinsics columns couple every frame: S is dense (k_cholesky_global: arrowhead)
      panel_bend[pk] = std::min(jmax, 6 * NB_);
      panel_jmax[pk] = n_;
    }
  }
  if (nk_) panel_jmax.insert(panel_jmax.end(), panel_bend.begin(), panel_bend.end());   // work_i_ tail
  {
    std::vector<int32_t> off(npanel + 1, 0);
    for (int pk = 0; pk < npanel; ++pk)
      off[pk + 1] = off[pk] + std::min(kCholNb, n_ - pk * kCholNb) * (panel_jmax[pk] - pk * kCholNb);
    npack_ = (size_t)off[npanel] + n_;
    stager_->Add(pack_off_, off);
    // + the merged exchange's tail (k_cam_finalize modes 1, 2)
    ntail_ = 2 * (size_t)6 * NB_ + kXNum + nranks() + 1;
    Spk_.Resize(npack_ + ntail_);
  }
  // k_cholesky_global stages each panel's rows in LDS when x and 16 rows of S fit
  // (SG_CHOL_GSTAGE=0: never, so tests reach the unstaged instance at any size)
  chol_gstage_ = (size_t)std::max(n_, 1) * 8 * (1 + kCholNb) <= gchol_lds_max_ &&
                 !(getenv("SG_CHOL_GSTAGE") && atoi(getenv("SG_CHOL_GSTAGE")) == 0);
  chol_window_ = npanel <= kJendSh;   // band ends cached in LDS
  for (int pk = 0; pk < npanel; ++pk)
    if (panel_jmax[pk] - pk * kCholNb > kCholWS) chol_window_ = false;
  band_tiles_ = 0;
  for (int pk = 0; pk < npanel; ++pk)
    band_tiles_ = std::max(band_tiles_, (panel_jmax[pk] + kCholNb - 1) / kCholNb - pk);
  // tiled band Cholesky: every tile row's band within kTB tiles, x and z' of the whole system in LDS
  chol_tiles_ = n_ > 0 && nk_ == 0 && npanel <= kTileMaxNT && !getenv("SG_CHOL_WINDOW");
  for (int pk = 0; pk < npanel; ++pk)
    if ((panel_jmax[pk] + kCholNb - 1) / kCholNb - pk > kTB) chol_tiles_ = false;
  // free intrinsics (one 16-wide border tile): the frame band on k_chol_tiles, the border by k_chol_border
  // (SG_CHOL_BORDER=0: the arrowhead k_cholesky_global)
  chol_border_ = false;
  if (nk_ > 0 && NB_ > 0 && n_ - 6 * NB_ <= kCholNb && !getenv("SG_CHOL_WINDOW") &&
      !(getenv("SG_CHOL_BORDER") && atoi(getenv("SG_CHOL_BORDER")) == 0)) {
    const int ntf = (6 * NB_ + kCholNb - 1) / kCholNb;
    chol_border_ = ntf <= kTileMaxNT;
    for (int pk = 0; pk < ntf; ++pk)
      if ((panel_bend[pk] + kCholNb - 1) / kCholNb - pk > kTB) chol_border_ = false;
    if (chol_border_) {
      chol_tiles_ = true;
      // q_K tiles and the candidate operands in LDS where they fit (else global q_K / chol_candidates)
      border_flags_ = 0;
      for (int f : {1, 2, 3})   // the last that fits: both, else the candidate operands, else the q_K tiles
        if (border_lds_doubles(ntf, f, F_, D_, n_) * sizeof(double) <= border_lds_max_ &&
            (!(f & 2) || (F_ <= kCandMax && D_ <= kCandMax)))
          border_flags_ = f;
    }
  }
  // dissected band: a second workgroup factors the bottom nd tile rows (reversed) while the first factors
  // the top rows [0, m), both meeting at a separator of ns <= 7 tile rows (k_chol_tiles); worth it from about 12
  // tile rows.  The separator must hold every band of the top part: ns(m) = max_{K<m} tend[K] - m.  The chain is
  // priced in phases as max(m, nd + h) + ns, h = 2.5 phases for the bottom's hand-off (round-2 stamps: nd = 3 / 4 /
  // 5 at ns = 7 took 198 / 188 / 193 k cycles at C2), and the cheapest m is taken (C2, whose rows are 6-7 tiles
  // wide: m = 7, ns = 5, nd = 6 — 12 phases on the top chain instead of 14; C5, 8 tiles: ns = 7, nd = 33 as before).
  // SG_CHOL_SEP=7: the fixed 7-row separator (tests).
  chol_nd_ = 0;
  chol_ns_ = kTB - 1;
  if (chol_tiles_ && !chol_border_ && npanel >= kSplitMinNT &&
      !(getenv("SG_CHOL_SPLIT") && atoi(getenv("SG_CHOL_SPLIT")) == 0)) {
    const bool fixed7 = getenv("SG_CHOL_SEP") && atoi(getenv("SG_CHOL_SEP")) == kTB - 1;
    double best = 1e30;
    int reach = 0;   // max_{K<m} tend[K]
    for (int m = 1; m < npanel; ++m) {
      reach = std::max(reach, std::min(npanel, (panel_jmax[m - 1] + kCholNb - 1) / kCholNb));
      const int ns = fixed7 ? kTB - 1 : reach - m;
      const int nd = npanel - m - ns;
      if (ns < 1 || ns > kTB - 1 || reach - m > ns || nd < 2) continue;
      const double cost = std::max((double)m, nd + 2.5) + ns;
      if (cost < best) {
        best = cost;
        chol_nd_ = nd;
        chol_ns_ = ns;
      }
    }
  }
  if (chol_tiles_) {
    // W tiles of the top and bottom halves, the bottom's z' (+ failure slot), the separator contribution
    // and its rhs, then the constants {0, 1}
    // (zeroed and its constants set on the device by ResetState: no host fill, no staged zeros)
    Wg_.Resize((size_t)2 * npanel * kTB * 256 + 16 * (size_t)npanel + 49 * 256 + 7 * 16 + 2);
    stager_->Add(tflag_, std::vector<int32_t>(2, 0));
    tile_lds_ = (size_t)npanel * 32 * sizeof(double) + (size_t)(3 * npanel + 1) / 2 * sizeof(double);
    chol_cand_lds_ = !chol_border_ && F_ <= kCandMax && D_ <= kCandMax &&
                     tile_lds_ + cand_lds_bytes(F_, D_, n_) <= 100 * 1024 &&
                     tile_lds_ + cand_lds_bytes(F_, D_, n_) <= tile_lds_set_;
    if (chol_cand_lds_) tile_lds_ += cand_lds_bytes(F_, D_, n_);
    if (tile_lds_ > tile_lds_set_) {   // beyond the LDS granted at construction: the one-workgroup kernels
      chol_tiles_ = false;
      chol_border_ = false;
      chol_nd_ = 0;
    }
  }
  // k_S_reduce work: the band tiles (R <= C) of the frame columns, and per tile the segment tiles covering it
  // (segment order).  A segment tile outside the band is zero (no point couples its rows and columns).
  std::vector<int32_t> stile, s_loff, s_lidx;
  {
    const int nft = (6 * NB_ + kCholNb - 1) / kCholNb;
    std::vector<int32_t> row_off(nft + 1, 0), cend(nft, 0);
    for (int R = 0; R < nft; ++R) {
      cend[R] = std::min(nft, (panel_jmax[R] + kCholNb - 1) / kCholNb);
      row_off[R + 1] = row_off[R] + std::max(0, cend[R] - R);
      for (int C = R; C < cend[R]; ++C) stile.push_back((R << 16) | C);
    }
    std::vector<std::vector<int32_t>> tl(stile.size());
    for (const SchurSeg& sg : segs)
      for (int u = 0; u < sg.ntw * (sg.ntw + 1) / 2; ++u) {
        const int R = sg.t0 + schur_tile_r(u), C = sg.t0 + schur_tile_c(u);
        if (R < nft && C < cend[R]) tl[row_off[R] + C - R].push_back(sg.s_off + 256 * u);
      }
    size_t smax = 0;
    for (const auto& l : tl) smax = std::max(smax, l.size());
    s_lstride_ = (int)std::max<size_t>(256, (smax + 255) / 256 * 256);   // rows padded (k_S_reduce's unbounded reads)
    s_lidx.assign(std::max<size_t>(tl.size(), 1) * s_lstride_, 0);
    for (size_t t = 0; t < tl.size(); ++t) {
      s_loff.push_back((int)tl[t].size());
      std::copy(tl[t].begin(), tl[t].end(), s_lidx.begin() + t * s_lstride_);
    }
    nstile_ = (int)stile.size();
    if (stile.empty()) stile.push_back(0);
    if (s_loff.empty()) s_loff.push_back(0);
  }
  lap("envelope");
  // upload batch 2 — the work lists: one pinned staging copy and one scatter launch (stager.h)
  stg.Add(lchunks_d_, lchunks);
  stg.Add(lrounds_d_, lrounds);
  stg.Add(segs_, segs.empty() ? std::vector<SchurSeg>(1) : segs);
  stg.Add(sbatch_, sbatch.empty() ? std::vector<SchurBatch>(1) : sbatch);
  stg.Add(wsegs_, wsegs.empty() ? std::vector<WideSeg>(1) : wsegs);
  stg.Add(pinfo_, pinfo);
  stg.Add(pmx_, pmx);
  stg.Add(cells_, cells);
  stg.Add(cell_obs_, cell_obs);
  stg.Add(stile_, stile);
  stg.Add(pairs_, pairs_flat);
  seg_fail_.Resize(std::max(nseg_ + nwide_, 1));
  stg.Add(cam_loff_, cam_loff);
  stg.Add(cam_lidx_, cam_lidx);
  stg.Add(s_loff_, s_loff);
  stg.Add(s_lidx_, s_lidx);
  stg.Add(r_loff_, r_loff);
  stg.Add(r_lidx_, r_lidx);
  // padded to one entry: k_cam_finalize prefetches fd_a[0] / fd_b[0] beside LmState even when D = 0
  stg.Add(fd_a_, fd_a.empty() ? std::vector<int32_t>{0} : fd_a);
  stg.Add(fd_b_, fd_b.empty() ? std::vector<int32_t>{0} : fd_b);
  stg.Add(fd_boff_, fd_boff);
  stg.Add(fd_bidx_, fd_bidx.empty() ? std::vector<int32_t>{0} : fd_bidx);
  stg.Add(work_i_, panel_jmax);
  {
    // FrameDistance cross-block lookup for the on-the-fly assembly: fd_pair[I*NB+J] (I<J) = 2 * residual +
    // (1 if the residual's frame a is block J, not I), so k_S_reduce reads the orientation with the index
    // instead of two more dependent loads (fd_a, frame_block)
    std::vector<int32_t> fd_pair((size_t)std::max(NB_, 1) * std::max(NB_, 1), -1);
    for (int dd = 0; dd < D_; ++dd) {
      const int ba = frame_block[fd_a[dd]], bb = frame_block[fd_b[dd]];
      if (ba >= 0 && bb >= 0 && ba != bb)
        fd_pair[(size_t)std::min(ba, bb) * NB_ + std::max(ba, bb)] = 2 * dd + (ba < bb ? 0 : 1);
    }
    stg.Add(fd_pair_, fd_pair);
    rdg_.Resize((size_t)std::max(n_, 1) + kCholNb);   // + padding rows of the last panel
  }
  // the linearization's buffers hold two slots (current point, k_update_lin's candidate)
  jslot_ = (size_t)((std::max(M_, 1) + 63) & ~63) * kJStride;   // whole 64-observation blocks (jidx2)
  J_.Resize(2 * jslot_);
  V_.Resize(2 * 10 * (size_t)std::max(P_, 1));
  g_.Resize(2 * 4 * (size_t)std::max(P_, 1));
  scale_p_.Resize(4 * (size_t)std::max(P_, 1));
  diag_p_.Resize(4 * (size_t)std::max(P_, 1));
  Vinv_.Resize(10 * (size_t)std::max(P_, 1));
  tp_.Resize(4 * (size_t)std::max(P_, 1));
  const size_t nn = std::max(n_, 1);
  scale_c_.Resize(nn);
  diag_c_.Resize(nn);
  camdiag_.Resize(nn);
  camg_.Resize(nn);
  cslot_ = std::max(lcam_off, 1);
  cam_slab_.Resize(2 * cslot_);
  lin_scal_.Resize(2 * (size_t)std::max(nlin_, 1) * kNScal);
  S_slab_.Resize(std::max(s_off, 1));
  chunk_scal_.Resize((size_t)std::max(npu_, 1) * kNScal);
  stg.Add(pu_units_, pu_units);
  if (nk_) {
    // free intrinsics: each frame block's non-fixed observations (block NB: the fixed frames'), for k_intr_fk
    std::vector<int32_t> boff(NB_ + 2, 0), bidx;
    for (int o = 0; o < M_; ++o)
      if (!(obs_meta[o] & kMetaFixed)) {
        const int b = meta_block(obs_meta[o]);
        boff[(b >= 0 ? b : NB_) + 1] += 1;
      }
    for (int b = 0; b <= NB_; ++b) boff[b + 1] += boff[b];
    bidx.resize(std::max(boff[NB_ + 1], 1), 0);
    std::vector<int32_t> fill(boff.begin(), boff.end() - 1);
    for (int o = 0; o < M_; ++o)
      if (!(obs_meta[o] & kMetaFixed)) {
        const int b = meta_block(obs_meta[o]);
        bidx[fill[b >= 0 ? b : NB_]++] = o;
      }
    stg.Add(intr_boff_, boff);
    stg.Add(intr_bidx_, bidx);
    // slices per block list: about one observation per thread of a k_intr_fk workgroup
    int lmax = 1;
    for (int b = 0; b <= NB_; ++b) lmax = std::max(lmax, boff[b + 1] - boff[b]);
    intr_nsl_ = std::max(1, std::min(32, (lmax + 255) / 256));
  }
  if (host_timing) DevMark(s, 1);
  stg.Flush(s);
  if (host_timing) DevMark(s, 2);
  lap("flush");
  cam_wide_.Resize(2 * (size_t)std::max(NB_, 1) * kCamV);
  S_wide_.Resize(nn * nn);
  zpre_.Resize(257);
  xchg_cam_.Resize(3 * ((size_t)NB_ * kCamV + kXNum + nranks()));   // summed | this rank's | candidate
  S_.Resize(nn * nn + nn + 2);   // S, then the rhs partial xc (one all-reduce covers both), then {0, 1}
  rhs_.Resize(nn);
  xchg_upd_.Resize(kUNum);
  xchg_chol_.Resize(kCNum);
  work_.Resize(nn);
  fd_r_.Resize(std::max(D_, 1));
  fd_J_.Resize(6 * (size_t)std::max(D_, 1));
  fd_D_.Resize(9 * (size_t)std::max(NB_, 1));
  fd_X_.Resize(9 * (size_t)std::max(D_, 1));
  if (nk_) {
    Jk_.Resize(14 * (size_t)std::max(M_, 1));
    KU_.Resize(nn * nk_);
    kst_.Resize(56 * (size_t)ncam_);
    Yk_.Resize(28 * (size_t)std::max(P_, 1) * ncam_);
    kpart_.Resize((size_t)(NB_ + 1) * ncam_ * 42);
  }
  stamp_on_ = getenv("SG_STAMP") && getenv("SG_STAMP")[0] == '1';
  if (stamp_on_) stamps_.Resize(kSegStamp + 8 * kSegStampMax);
  lap("resize");
  ResetState(s);
  if (host_timing) DevMark(s, 3);
  lap("reset");
  WaitStream(s);
  lap("uploads");
  if (host_timing) {
    float a = 0, b = 0, c = 0;
    (void)hipEventElapsedTime(&a, dev_marks_[0], dev_marks_[1]);
    (void)hipEventElapsedTime(&b, dev_marks_[1], dev_marks_[2]);
    (void)hipEventElapsedTime(&c, dev_marks_[2], dev_marks_[3]);
    float e = 0;
    (void)hipEventElapsedTime(&e, dev_marks_[4], dev_marks_[3]);
    const double hw = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - load_t0).count();
    char buf[320];
    snprintf(buf, sizeof(buf), " [device: batch1..batch2 %.2f, scatter2 %.2f, reset %.2f; load start..reset: device "
             "%.2f, host %.2f]", a, b, c, e, hw);
    lap_log += buf;
    if (idle_valid_prev) {
      float g = 0;
      const hipError_t ge = hipEventElapsedTime(&g, ev_idle_prev_, dev_marks_[4]);
      snprintf(buf, sizeof(buf), " [last idle..load start: device %.2f (%d), host %.2f]", g, (int)ge, idle_gap_host);
      lap_log += buf;
    }
  }
  if (host_timing) {
    char buf[96];
    snprintf(buf, sizeof(buf), " (staged %.2f MB; device allocations so far %ld)", stg.staged_bytes() / 1e6,
             g_dbuf_allocs.load());
    lap_log += buf;
  }
  SaveStructure(p);
  full_loads_++;
  if (host_timing) {
    SG_HIP_CHECK(hipStreamSynchronize(stream_));
    lap("sync");
    fprintf(stderr, "[sg] Load phases (ms):%s\n", lap_log.c_str());
  }
  loaded_ = true;
  began_ = false;
  pending_decision_ = false;
}

void BaSolver::Reserve(int F, int P, int M) {
  SG_REQUIRE(F >= 0 && P >= 0 && M >= 0, SG_EINVAL, "negative reservation");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  const size_t f = std::max(F, 1), pp = std::max(P, 1), m = std::max(M, 1);
  bool moved = false;
  // per observation (device order records, the Jacobian rows, the Schur cells)
  moved |= J_.Reserve(2 * ((m + 63) & ~(size_t)63) * kJStride);
  moved |= obs_pt_.Reserve(2 * m);
  moved |= obs_frame_.Reserve(m);
  moved |= obs_fixed_.Reserve(m);
  moved |= obs_meta_.Reserve(m);
  moved |= obs_pnt_.Reserve(m);
  moved |= cells_.Reserve(4 * m);
  moved |= cell_obs_.Reserve(m);
  // per point
  moved |= X_.Reserve(8 * pp);
  moved |= V_.Reserve(2 * 10 * pp);
  moved |= Vinv_.Reserve(10 * pp);
  moved |= g_.Reserve(2 * 4 * pp);
  moved |= tp_.Reserve(4 * pp);
  moved |= scale_p_.Reserve(4 * pp);
  moved |= diag_p_.Reserve(4 * pp);
  moved |= pfree_.Reserve(pp);
  moved |= poff_.Reserve(pp + 1);
  moved |= pinfo_.Reserve(2 * pp);
  moved |= pmx_.Reserve(4 * pp);
  // per frame
  moved |= q_.Reserve(8 * f);
  moved |= t_.Reserve(6 * f);
  moved |= frame_cam_.Reserve(f);
  moved |= frame_block_.Reserve(f);
  moved |= rot_free_.Reserve(f);
  moved |= trans_free_.Reserve(f);
  // the pinned staging buffer and its device copy: about 51 B per observation, 93 B per point, and per frame
  // the pose slots, the FrameDistance pair table (NB^2) and the Cholesky's W tiles (2 * 8 tiles per 16 columns)
  moved |= stager_->ReserveBytes(64 * m + 128 * pp + 16384 * f + 4 * f * f + (1u << 20));
  if (moved) {   // the buffers of the loaded structure are gone: the next Load rebuilds everything
    loaded_ = false;
    began_ = false;
    skey_ = StructKey{};
  }
}

bool BaSolver::SameStructure(const sg_problem& p) const {
  const StructKey& k = skey_;
  if (p.num_cameras != k.ncam || (p.cameras_free != 0) != (k.cams_free != 0) || p.num_frames != k.F ||
      p.num_points != k.P || p.num_obs != k.M || p.num_dist != k.D)
    return false;
  auto same = [](const auto* a, const auto& v) {
    return v.empty() || std::memcmp(a, v.data(), v.size() * sizeof(v[0])) == 0;
  };
  return same(p.frame_camera, k.frame_camera) && same(p.frame_rot_free, k.rot_free) &&
         same(p.frame_trans_free, k.trans_free) && same(p.point_free, k.point_free) &&
         same(p.obs_frame, k.obs_frame) && same(p.obs_point, k.obs_point) && same(p.dist_frame, k.dist_frame) &&
         same(p.dist_prev, k.dist_prev);
}

void BaSolver::SaveStructure(const sg_problem& p) {
  StructKey& k = skey_;
  k.ncam = p.num_cameras;
  k.cams_free = p.cameras_free != 0;
  k.F = p.num_frames;
  k.P = p.num_points;
  k.M = p.num_obs;
  k.D = p.num_dist;
  k.frame_camera.assign(p.frame_camera, p.frame_camera + k.F);
  k.rot_free.assign(p.frame_rot_free, p.frame_rot_free + k.F);
  k.trans_free.assign(p.frame_trans_free, p.frame_trans_free + k.F);
  k.point_free.assign(p.point_free, p.point_free + k.P);
  k.obs_frame.assign(p.obs_frame, p.obs_frame + k.M);
  k.obs_point.assign(p.obs_point, p.obs_point + k.M);
  k.dist_frame.assign(p.dist_frame, p.dist_frame + k.D);
  k.dist_prev.assign(p.dist_prev, p.dist_prev + k.D);
}

// LM state and accumulators a fresh solve starts from (zeroed on every Load)
// Zero a few device buffers and set the tiled Cholesky's {0, 1} constants (after S and its rhs) in one launch
// (hipMemsetAsync / a pageable hipMemcpyAsync would go through the copy engine).
constexpr int kZeroBufs = 9;
struct ZeroList {
  double* p[kZeroBufs];
  size_t n[kZeroBufs];   // doubles
  double* c01[2];        // two doubles each: {0, 1}
};
__global__ __launch_bounds__(256) void k_reset_buffers(ZeroList z) {
  for (int b = 0; b < kZeroBufs; ++b) {
    double* p = z.p[b];
    const size_t n = z.n[b];
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      p[i] = 0.0;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2 && z.c01[threadIdx.x]) {
    z.c01[threadIdx.x][0] = 0.0;
    z.c01[threadIdx.x][1] = 1.0;
  }
}

void BaSolver::ResetState(hipStream_t s) {
  // LmState (slot 0 current, nothing pending: evaluate() may run before begin()), the accumulators, S; one
  // launch, no copy engine (hostmirror.h)
  ZeroList z{};
  auto put = [&](int i, void* ptr, size_t bytes) {
    z.p[i] = static_cast<double*>(ptr);
    z.n[i] = ptr ? bytes / 8 : 0;
  };
  static_assert(sizeof(LmState) % 8 == 0, "LmState is zeroed in 8-byte words");
  put(0, st_.ptr, st_.size * sizeof(LmState));
  put(1, lin_scal_.ptr, lin_scal_.size * sizeof(double));
  put(2, seg_fail_.ptr, seg_fail_.size * sizeof(*seg_fail_.ptr));
  put(3, cam_wide_.ptr, cam_wide_.size * sizeof(double));
  put(4, S_wide_.ptr, S_wide_.size * sizeof(double));
  put(5, rhs_.ptr, rhs_.size * sizeof(double));
  put(6, chunk_scal_.ptr, chunk_scal_.size * sizeof(double));
  put(7, S_.ptr, (S_.size - 2) * sizeof(double));
  z.c01[0] = S_.ptr + S_.size - 2;   // k_chol_tiles: padding entries of the last tile
  if (chol_tiles_ && Wg_.size >= 2) {   // its W tiles, z', separator terms, then its own {0, 1}
    put(8, Wg_.ptr, (Wg_.size - 2) * sizeof(double));
    z.c01[1] = Wg_.ptr + Wg_.size - 2;
  }
  size_t mx = 0;
  for (int i = 0; i < kZeroBufs; ++i) mx = std::max(mx, z.n[i]);
  const unsigned g = (unsigned)std::min<size_t>(512, std::max<size_t>(1, (mx + 255) / 256));
  hipLaunchKernelGGL(k_reset_buffers, dim3(g), dim3(256), 0, s, z);
  SG_HIP_CHECK(hipGetLastError());
  if (stamp_on_) stamps_.Zero(s);
}

// Same structure as the last Load: new values (poses, intrinsics, points, observed pixels, loss ranges) in
// the device order of that Load; every index list and the Cholesky envelope stay.
void BaSolver::LoadValues(const sg_problem& p) {
  range_b_ = p.range * p.range;
  fd_target_ = p.dist_target;
  fd_b2_ = p.dist_range * p.dist_range;
  stab_b_ = p.stab_range * p.stab_range;
  hipStream_t s = stream_;
  std::vector<double> k2(14 * (size_t)ncam_), q2(8 * (size_t)F_), t2(6 * (size_t)F_), X2(8 * (size_t)P_),
      obs_pt(2 * (size_t)M_);
  for (int c = 0; c < 7 * ncam_; ++c) k2[c] = k2[c + 7 * ncam_] = p.k[c];
  for (int i = 0; i < 4 * F_; ++i) q2[i] = q2[i + 4 * F_] = p.q[i];
  for (int i = 0; i < 3 * F_; ++i) t2[i] = t2[i + 3 * F_] = p.t[i];
  for (int i = 0; i < P_; ++i) {
    const int pt = point_perm_[i];
    for (int a = 0; a < 4; ++a) X2[4 * i + a] = X2[4 * (i + P_) + a] = p.X[4 * pt + a];
  }
  for (int o = 0; o < M_; ++o) {
    const int src = obs_perm_[o];
    obs_pt[2 * o] = p.obs_pt[2 * src];
    obs_pt[2 * o + 1] = p.obs_pt[2 * src + 1];
  }
  k_.Upload(k2.empty() ? std::vector<double>{0.0} : k2, s);
  q_.Upload(q2, s);
  t_.Upload(t2, s);
  X_.Upload(X2, s);
  obs_pt_.Upload(obs_pt, s);
  ResetState(s);
  SG_HIP_CHECK(hipStreamSynchronize(s));
  value_loads_++;
  loaded_ = true;
  began_ = false;
  pending_decision_ = false;
}

Dev BaSolver::MakeDev() {
  Dev d{};
  d.st = st_.ptr;
  d.k[0] = k_.ptr;
  d.k[1] = k_.ptr + 7 * (size_t)ncam_;
  d.nk = nk_;
  d.kc0 = 6 * NB_;
  d.ncam = ncam_;
  d.Jk = Jk_.ptr;
  d.KU = KU_.ptr;
  d.kst = kst_.ptr;
  d.Yk = Yk_.ptr;
  d.kpart = kpart_.ptr;
  d.intr_boff = intr_boff_.ptr;
  d.intr_bidx = intr_bidx_.ptr;
  d.stab_b = stab_b_;
  d.stab_inv_b = 1.0 / stab_b_;
  d.q[0] = q_.ptr;
  d.q[1] = q_.ptr + 4 * (size_t)F_;
  d.t[0] = t_.ptr;
  d.t[1] = t_.ptr + 3 * (size_t)F_;
  d.frame_cam = frame_cam_.ptr;
  d.frame_block = frame_block_.ptr;
  d.rot_free = rot_free_.ptr;
  d.trans_free = trans_free_.ptr;
  d.F = F_;
  d.NB = NB_;
  d.n = n_;
  d.X[0] = X_.ptr;
  d.X[1] = X_.ptr + 4 * (size_t)P_;
  d.pfree = pfree_.ptr;
  d.poff = poff_.ptr;
  d.P = P_;
  d.M = M_;
  d.obs_pt = obs_pt_.ptr;
  d.obs_frame = obs_frame_.ptr;
  d.obs_fixed = obs_fixed_.ptr;
  d.obs_meta = obs_meta_.ptr;
  d.b = range_b_;
  d.inv_b = 1.0 / range_b_;
  d.D = D_;
  d.fd_a = fd_a_.ptr;
  d.fd_b = fd_b_.ptr;
  d.fd_boff = fd_boff_.ptr;
  d.fd_bidx = fd_bidx_.ptr;
  d.fd_target = fd_target_;
  d.fd_b2 = fd_b2_;
  d.fd_inv_b2 = 1.0 / fd_b2_;
  d.fd_r = fd_r_.ptr;
  d.fd_J = fd_J_.ptr;
  d.fd_D = fd_D_.ptr;
  d.fd_X = fd_X_.ptr;
  {
    const size_t pp = std::max(P_, 1);
    for (int sl = 0; sl < 2; ++sl) {
      d.J[sl] = J_.ptr + sl * jslot_;
      d.V[sl] = V_.ptr + sl * 10 * pp;
      d.g[sl] = g_.ptr + sl * 4 * pp;
      d.cam_slab[sl] = cam_slab_.ptr + sl * cslot_;
      d.cam_wide[sl] = cam_wide_.ptr + sl * (size_t)std::max(NB_, 1) * kCamV;
      d.lin_scal[sl] = lin_scal_.ptr + sl * (size_t)std::max(nlin_, 1) * kNScal;
    }
  }
  d.spec = spec_ ? 1 : 0;
  d.scale_p = scale_p_.ptr;
  d.diag_p = diag_p_.ptr;
  d.Vinv = Vinv_.ptr;
  d.tp = tp_.ptr;
  d.scale_c = scale_c_.ptr;
  d.diag_c = diag_c_.ptr;
  d.camdiag = camdiag_.ptr;
  d.camg = camg_.ptr;
  d.cam_loff = cam_loff_.ptr;
  d.cam_lidx = cam_lidx_.ptr;
  d.s_loff = s_loff_.ptr;
  d.s_lidx = s_lidx_.ptr;
  d.r_loff = r_loff_.ptr;
  d.r_lidx = r_lidx_.ptr;
  d.s_lstride = s_lstride_;
  d.r_lstride = r_lstride_;
  d.S_slab = S_slab_.ptr;
  d.chunk_scal = chunk_scal_.ptr;
  d.S_wide = S_wide_.ptr;
  d.zpre = zpre_.ptr;
  d.xchg_cam = xchg_cam_.ptr;
  d.xcam_loc = xchg_cam_.ptr + (size_t)NB_ * kCamV + kXNum + nranks();
  d.xchg_cand = xchg_cam_.ptr + 2 * ((size_t)NB_ * kCamV + kXNum + nranks());
  d.xtail = Spk_.ptr + npack_;
  d.rank = comm_ ? comm_->rank() : 0;
  d.nranks = nranks();
  d.S = S_.ptr;
  d.rhs = rhs_.ptr;
  d.xchg_upd = xchg_upd_.ptr;
  d.xchg_chol = xchg_chol_.ptr;
  d.xc = S_.ptr + (size_t)n_ * n_;
  d.work = work_.ptr;
  d.stamps = stamp_on_ ? stamps_.ptr : nullptr;
  d.fd_pair = fd_pair_.ptr;
  d.obs_pnt = obs_pnt_.ptr;
  d.lchunks = lchunks_d_.ptr;
  d.lrounds = lrounds_d_.ptr;
  d.nlin = nlin_;
  d.npu = npu_;
  d.pu_units = pu_units_.ptr;
  d.segs = segs_.ptr;
  d.nseg = nseg_;
  d.sbatch = sbatch_.ptr;
  d.pinfo = reinterpret_cast<const int2*>(pinfo_.ptr);
  d.pmx = reinterpret_cast<const int4*>(pmx_.ptr);
  d.cells = reinterpret_cast<const int4*>(cells_.ptr);
  d.cell_obs = cell_obs_.ptr;
  d.wsegs = wsegs_.ptr;
  d.nwide = nwide_;
  d.stile = stile_.ptr;
  d.nstile = nstile_;
  d.seg_fail = seg_fail_.ptr;
  d.pairs = reinterpret_cast<const int2*>(pairs_.ptr);
  d.assemble = (!comm_ || comm_->rank() == 0) ? 1 : 0;
  return d;
}

// The LM state handed over as a kernel argument (no host buffer, no copy engine: see hostmirror.h).
__global__ void k_set_state(LmState s, LmState* st) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *st = s;
}

// The current parameter slot's poses, points and intrinsics into the mapped download buffer
// [q 4F | t 3F | X 4P | k 7 ncam] (the slot is read on the device: no state round trip first).
__global__ __launch_bounds__(256) void k_download(const double* __restrict__ q, const double* __restrict__ t,
                                                  const double* __restrict__ X, const double* __restrict__ k,
                                                  const LmState* st, int F, int P, int ncam, double* __restrict__ out) {
  const int cur = st->cur;
  const size_t nq = 4 * (size_t)F, nt = 3 * (size_t)F, nx = 4 * (size_t)P, nk = 7 * (size_t)ncam;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq + nt + nx + nk;
       i += (size_t)gridDim.x * blockDim.x) {
    double v;
    if (i < nq) v = q[nq * cur + i];
    else if (i < nq + nt) v = t[nt * cur + (i - nq)];
    else if (i < nq + nt + nx) v = X[nx * cur + (i - nq - nt)];
    else v = k[nk * cur + (i - nq - nt - nx)];
    out[i] = v;
  }
}

// Wait for stream s by spinning on an event query.  hipStreamSynchronize's blocking wait returned 13-28 ms
// late in a few percent of the main.cpp replay's loads, all of whose work had been three small kernels
// (tools/e2e_replay.py, profiles/r3_v8_*); the solver's waits are short (a load, an LM batch), so the host
// spins on them, falling back to the blocking wait after 200 ms.  A sharded solver (several
// ranks, possibly rank threads or processes sharing the host's cores with the threads that run the host
// all-reduces) yields between polls and spins at most 1 ms.
void BaSolver::WaitStream(hipStream_t s) {
  constexpr double spin_ms = 200.0;
  const bool shared = nranks() > 1;
  const double limit = shared ? std::min(spin_ms, 1.0) : spin_ms;
  if (!ev_wait_) SG_HIP_CHECK(hipEventCreateWithFlags(&ev_wait_, hipEventDisableTiming));
  SG_HIP_CHECK(hipEventRecord(ev_wait_, s));
  const auto t0 = std::chrono::steady_clock::now();
  while (true) {
    const hipError_t e = hipEventQuery(ev_wait_);
    if (e == hipSuccess) {
      MarkIdle(s);
      return;
    }
    if (e != hipErrorNotReady) SG_HIP_CHECK(e);
    if (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > limit) break;
    if (shared) std::this_thread::yield();
  }
  SG_HIP_CHECK(hipEventSynchronize(ev_wait_));
  MarkIdle(s);
}

// SG_HOST_TIMING: a device marker and the host clock at the moment the stream was last seen idle, so a load can
// compare the device's and the host's time from there to its first command (a late queue start shows as a
// device gap longer than the host's).
void BaSolver::MarkIdle(hipStream_t s) {
  static const bool host_timing = getenv("SG_HOST_TIMING") != nullptr;
  if (!host_timing) return;
  if (!ev_idle_) SG_HIP_CHECK(hipEventCreate(&ev_idle_));
  SG_HIP_CHECK(hipEventRecord(ev_idle_, s));
  idle_host_ = std::chrono::steady_clock::now();
  idle_valid_ = true;
}

void BaSolver::DevMark(hipStream_t s, int i) {
  if (!dev_marks_[i]) SG_HIP_CHECK(hipEventCreate(&dev_marks_[i]));
  SG_HIP_CHECK(hipEventRecord(dev_marks_[i], s));
}

void BaSolver::ReadState(LmState* h) {
  static_assert(sizeof(LmState) % 8 == 0, "LmState is copied in 8-byte words");
  mb_.Reserve(1024);
  hipLaunchKernelGGL(k_copy_u64, dim3(1), dim3(64), 0, stream_, reinterpret_cast<const unsigned long long*>(st_.ptr),
                     reinterpret_cast<unsigned long long*>(mb_.d), sizeof(LmState) / 8);
  WaitStream(stream_);
  std::memcpy(h, mb_.h, sizeof(LmState));
}

void BaSolver::Begin(const sg_solver_options& o) {
  SG_REQUIRE(loaded_, SG_EINVAL, "no problem loaded");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  const bool began_again = began_;
  if (began_) {
    // restart from the current parameter slot: move it to slot 0 (a fresh load starts in slot 0: no round trip)
    LmState h{};
    ReadState(&h);
    if (h.cur == 1) {
      SG_HIP_CHECK(hipMemcpyAsync(q_.ptr, q_.ptr + 4 * (size_t)F_, 4 * (size_t)F_ * 8, hipMemcpyDeviceToDevice, stream_));
      SG_HIP_CHECK(hipMemcpyAsync(t_.ptr, t_.ptr + 3 * (size_t)F_, 3 * (size_t)F_ * 8, hipMemcpyDeviceToDevice, stream_));
      SG_HIP_CHECK(hipMemcpyAsync(X_.ptr, X_.ptr + 4 * (size_t)P_, 4 * (size_t)P_ * 8, hipMemcpyDeviceToDevice, stream_));
      if (ncam_ > 0)
        SG_HIP_CHECK(hipMemcpyAsync(k_.ptr, k_.ptr + 7 * (size_t)ncam_, 7 * (size_t)ncam_ * 8, hipMemcpyDeviceToDevice,
                                    stream_));
    }
  }
  began_ = true;
  LmState s{};
  s.max_iter = o.max_num_iterations;
  s.max_invalid = o.max_num_consecutive_invalid_steps;
  s.disable_term = o.disable_termination;
  s.always_lin = o.always_linearize;
  s.jacobi = o.jacobi_scaling;
  s.ftol = o.function_tolerance;
  s.gtol = o.gradient_tolerance;
  s.ptol = o.parameter_tolerance;
  s.min_rel_dec = o.min_relative_decrease;
  s.max_radius = o.max_trust_region_radius;
  s.min_radius = o.min_trust_region_radius;
  s.min_diag = o.min_lm_diagonal;
  s.max_diag = o.max_lm_diagonal;
  s.cur = 0;
  s.need_lin = 1;
  s.first = 1;
  s.done = (NB_ == 0 && P_ == 0) ? 1 : 0;
  s.ok = 1;
  s.termination = s.done ? SG_FUNCTION_TOLERANCE : SG_NO_CONVERGENCE;
  s.radius = o.initial_trust_region_radius;
  s.decrease_factor = 2.0;
  hipLaunchKernelGGL(k_set_state, dim3(1), dim3(64), 0, stream_, s, st_.ptr);
  if (began_again && spec_) {
    // k_cam_reduce keeps the wide-chunk camera accumulators in speculative mode: clear both slots for the
    // restart's first k_linearize (a fresh Load has zeroed them)
    ZeroList z{};
    z.p[0] = cam_wide_.ptr;
    z.n[0] = cam_wide_.size;
    hipLaunchKernelGGL(k_reset_buffers, dim3(1), dim3(256), 0, stream_, z);
  }
  need_seq_ = true;   // the first iteration fixes the camera scale: k_schur waits for it
  pending_decision_ = false;
  for (auto& t : timers_) {
    t.total_ms = 0.0;
    t.count = 0;
  }
}

void BaSolver::TimedLaunchBegin(int id) { TimedLaunchBegin(id, stream_); }
void BaSolver::TimedLaunchEnd(int id) { TimedLaunchEnd(id, stream_); }
void BaSolver::TimedLaunchBegin(int id, hipStream_t s) {
  if (!timing_) return;
  hipEvent_t a, b;
  SG_HIP_CHECK(hipEventCreate(&a));
  SG_HIP_CHECK(hipEventCreate(&b));
  timers_[id].ev.push_back(a);
  timers_[id].ev.push_back(b);
  SG_HIP_CHECK(hipEventRecord(a, s));
}
void BaSolver::TimedLaunchEnd(int id, hipStream_t s) {
  if (!timing_) return;
  SG_HIP_CHECK(hipEventRecord(timers_[id].ev.back(), s));
}

void BaSolver::Iterate(int n) {
  SG_REQUIRE(loaded_, SG_EINVAL, "no problem loaded");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  EnqueueIterations(n);
}

void BaSolver::EnqueueIterations(int n) {
  Dev d = MakeDev();
  for (int it = 0; it < n; ++it) {
    // speculative mode: only a solve's first iteration linearizes here; later ones find the linearization of
    // the accepted point in the slot k_update_lin filled (k_linearize would exit at once: no launch)
    if (!spec_ || need_seq_) {
      TimedLaunchBegin(kKLin);
      LaunchLinearize(d);
      TimedLaunchEnd(kKLin);
    }
    const bool first_it = need_seq_;
    need_seq_ = false;
    // Landmark shards exchange twice per LM iteration after a solve's first: k_S_reduce assembles each rank's
    // own camera blocks (and, on rank 0, the FrameDistance terms) into its partial S, and the camera gradient,
    // diagonal and cost scalars ride in the same all-reduce as the band of S (k_cam_finalize modes 1 and 2);
    // the first iteration sums the camera blocks first (the Jacobi scale of the camera columns comes from
    // them), then S.  SG_XCHG_MERGE=0: the three-exchange chain every iteration; =force: the merged chain on
    // one rank too (tests the path).
    const bool multi_x = (comm_ && comm_->nranks() > 1);
    const bool merged = !first_it && nk_ == 0 && (merge_ == 2 || (multi_x && merge_ == 1));
    const int nv = NB_ * kCamV;
    // Speculative chain: the previous iteration ended with the candidate's camera reduce and the update scalars
    // (k_cam_reduce mode 1, + their all-reduce on shards); the pending decision is taken by k_cam_finalize
    // itself (one rank, or merged shards), else by k_decide, which then also makes the accepted candidate's
    // blocks current.  No pending decision (a batch's first iteration: EnqueueIterations settles it at the
    // end of every batch): the current blocks are in place.
    // One rank (no free intrinsics): the previous iteration's reduce took the decision (k_cam_reduce mode 2) and
    // this iteration's finalize pass runs inside the k_schur launch.
    // Merged landmark shards (speculative chain): the pending decision as its own small launch (k_decide, which
    // also makes an accepted candidate's blocks current), the finalize pass's mode 1 inside the k_schur launch,
    // and its mode 2 inside the unpack after the band exchange (k_S_unpack_fin): two single-workgroup launches of
    // the replicated chain less per iteration.
    const bool fin_in_schur = spec_ && !first_it && !multi_x && nk_ == 0 && !merged;
    const bool fin1_in_schur = spec_ && merged;
    bool decide_in_fin = false;
    if (fin_in_schur) {
      // (nothing pending: the candidate blocks of an accepted step are taken by the pass)
    } else if (spec_ && !first_it) {
      if (pending_decision_) {
        decide_in_fin = nk_ == 0 && !fin1_in_schur && (merged || !multi_x);
        if (!decide_in_fin) {
          TimedLaunchBegin(kKDecide);
          LaunchDecideK(stream_, d, 1);
          TimedLaunchEnd(kKDecide);
        }
        pending_decision_ = false;
      }
    } else {
      TimedLaunchBegin(kKCamReduce);
      LaunchCamReduceK(NB_ + 1, stream_, d, 0);
      TimedLaunchEnd(kKCamReduce);
    }
    if (!merged) AllReduceSum(xchg_cam_.ptr, (size_t)nv + kXNum + nranks());
    if (nk_) {
      LaunchIntrLinearizeK(stream_, d, n_, nk_, NB_, ncam_, M_, intr_nsl_);
    }
    if (!fin_in_schur && !fin1_in_schur) {
      TimedLaunchBegin(kKCamFinal);
      LaunchCamFinalizeK(stream_, d, merged ? 1 : 0, decide_in_fin ? 1 : 0);
      TimedLaunchEnd(kKCamFinal);
    }
    TimedLaunchBegin(kKSchur);
    LaunchSchurK(std::max(nseg_, 1), nwide_, fin_in_schur ? 1 : (fin1_in_schur ? 2 : 0), stream_, d);
    TimedLaunchEnd(kKSchur);
    TimedLaunchBegin(kKSReduce);
    const int nwv = nstile_ + NB_;
    // S is final after k_S_reduce (one rank, no free intrinsics, no merged damping; a forced pack / unpack on one
    // rank is a copy): it also factors the first diagonal tile for k_chol_tiles (flags bit 4)
    const int samode = merged ? 2 : (d.assemble ? 1 : 0);
    const bool zpre = chol_tiles_ && !chol_border_ && nk_ == 0 && samode == 1 && !(multi_x || merged) && !chol_zpre_off_;
    LaunchSReduceK(std::max(nwv, 1), stream_, d, samode, zpre ? 1 : 0);
    TimedLaunchEnd(kKSReduce);
    if (nk_) {
      LaunchIntrSchurK(stream_, d, n_, nk_, NB_, ncam_, P_, intr_nsl_);
    }
    if (multi_x || pack_force_ || merged) {
      // the band of S and the rhs partial are summed over landmark shards (packed: the band only), with the
      // merged tail after them
      const int npanel = (n_ + kCholNb - 1) / kCholNb;
      const dim3 pg(npanel + 1, 4);
      TimedLaunchBegin(kKXchg);   // pack, all-reduce, unpack
      LaunchSPackK(pg, stream_, S_.ptr, n_, (const int32_t*)work_i_.ptr, (const int32_t*)pack_off_.ptr, npanel,
                   Spk_.ptr, 0);
      AllReduceSum(Spk_.ptr, npack_ + (merged ? ntail_ : 0));
      if (fin1_in_schur)
        LaunchSUnpackFinK(pg, stream_, d, (const int32_t*)work_i_.ptr, (const int32_t*)pack_off_.ptr, npanel,
                          Spk_.ptr);
      else
        LaunchSPackK(pg, stream_, S_.ptr, n_, (const int32_t*)work_i_.ptr, (const int32_t*)pack_off_.ptr, npanel,
                     Spk_.ptr, 1);
      TimedLaunchEnd(kKXchg);
      if (merged && !fin1_in_schur) {
        TimedLaunchBegin(kKCamFinal);
        LaunchCamFinalizeK(stream_, d, 2, 0);
        TimedLaunchEnd(kKCamFinal);
      }
    }
    TimedLaunchBegin(kKChol);
    if (chol_tiles_)
      LaunchCholTiles(d.stamps != nullptr, dim3(chol_nd_ > 0 ? 2 : 1), d,
                      (chol_cand_lds_ ? 2 : 0) | (chol_force_tmo_ ? 4 : 0) | (zpre ? 16 : 0));
    else if (chol_window_)
      LaunchCholWindowK(d.stamps != nullptr, stream_, d, (const int32_t*)work_i_.ptr, rdg_.ptr);
    else
      LaunchCholGlobalK(chol_gstage_, (size_t)std::max(n_, 1) * 8 * (chol_gstage_ ? 1 + kCholNb : 1), stream_, d,
                        (const int32_t*)work_i_.ptr, rdg_.ptr);
    TimedLaunchEnd(kKChol);
    if (nk_) LaunchIntrStepK(stream_, d);
    TimedLaunchBegin(kKPointUpd);
    if (spec_) {
      LaunchUpdateLin(d);
    } else {
      LaunchPointUpdateK(std::max(npu_, 1), stream_, d);
    }
    TimedLaunchEnd(kKPointUpd);
    const bool multi = comm_ && comm_->nranks() > 1;
    // the candidate's camera blocks and linearization scalars beside the update scalars, one launch; on one rank
    // (no free intrinsics, no forced merged chain) the decision too
    const bool decide_in_reduce = !multi && nk_ == 0 && merge_ != 2;
    TimedLaunchBegin(kKUpdRed);
    if (spec_)
      LaunchCamReduceK(NB_ + 2, stream_, d, decide_in_reduce ? 2 : 1);
    else
      LaunchUpdReduceK(stream_, d, multi ? 0 : 1);
    TimedLaunchEnd(kKUpdRed);
    if (multi) AllReduceSum(xchg_upd_.ptr, kUNum);
    if (spec_) {
      pending_decision_ = !decide_in_reduce;
    } else if (multi) {
      TimedLaunchBegin(kKDecide);
      LaunchDecideK(stream_, d, 0);
      TimedLaunchEnd(kKDecide);
    }
  }
  // a batch leaves no decision pending: the host's state reads and downloads see the decided step
  if (pending_decision_) {
    TimedLaunchBegin(kKDecide);
    LaunchDecideK(stream_, d, 1);
    TimedLaunchEnd(kKDecide);
    pending_decision_ = false;
  }
  SG_HIP_CHECK(hipGetLastError());
}

__global__ void k_force_linearize(LmState* st) {
  if (threadIdx.x == 0) {
    st->need_lin = 1;
    st->done = 0;
  }
}

void BaSolver::Sweep(int n) {
  SG_REQUIRE(loaded_, SG_EINVAL, "no problem loaded");
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  Dev d = MakeDev();
  for (int it = 0; it < n; ++it) {
    hipLaunchKernelGGL(k_force_linearize, dim3(1), dim3(64), 0, stream_, st_.ptr);
    TimedLaunchBegin(kKLin);
    LaunchLinearize(d);
    TimedLaunchEnd(kKLin);
  }
  SG_HIP_CHECK(hipGetLastError());
}

void BaSolver::LaunchLinearize(const Dev& d) { LaunchLinearizeK(lin_waves_, std::max(nlin_, 1), stream_, d); }

void BaSolver::LaunchUpdateLin(const Dev& d) {
  LaunchUpdateLinK(stamp_on_, lin_waves_, std::max(nlin_, 1), stream_, d);
}

std::vector<unsigned long long> BaSolver::Stamps() {
  std::vector<unsigned long long> v(stamp_on_ ? stamps_.size : 64, 0);
  if (!stamp_on_) return v;
  SG_HIP_CHECK(hipMemcpyAsync(v.data(), stamps_.ptr, v.size() * 8, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
  return v;
}

void BaSolver::Sync() { SG_HIP_CHECK(hipStreamSynchronize(stream_)); }

void BaSolver::Summary(sg_solver_summary* s) {
  LmState h{};
  ReadState(&h);
  std::memset(s, 0, sizeof(*s));
  s->num_iterations = h.pushed;
  s->num_successful_steps = h.n_succ;
  s->num_unsuccessful_steps = h.n_unsucc;
  s->num_invalid_steps = h.n_invalid;
  s->termination_type = h.termination;
  s->ok = h.ok;
  s->initial_cost = h.initial_cost;
  s->final_cost = h.min_pushed_cost + h.fixed_cost;
  s->fixed_cost = h.fixed_cost;
  s->trust_region_radius = h.radius;
  s->num_lm_iterations = h.lm_iters;
  s->sync_timeouts = h.sync_timeouts;
}

void BaSolver::Download(sg_problem* p) {
  const size_t nq = 4 * (size_t)F_, nt = 3 * (size_t)F_, nx = 4 * (size_t)P_, nk = nk_ ? 7 * (size_t)ncam_ : 0;
  const size_t tot = nq + nt + nx + nk;
  mb_.Reserve(1024 + 8 * std::max<size_t>(tot, 1));
  double* out_d = reinterpret_cast<double*>(mb_.d + 1024);
  const double* out = reinterpret_cast<const double*>(mb_.h + 1024);
  const unsigned g = (unsigned)std::min<size_t>(1024, std::max<size_t>(1, (tot + 255) / 256));
  hipLaunchKernelGGL(k_download, dim3(g), dim3(256), 0, stream_, q_.ptr, t_.ptr, X_.ptr, nk ? k_.ptr : q_.ptr,
                     (const LmState*)st_.ptr, F_, P_, nk ? ncam_ : 0, out_d);
  WaitStream(stream_);
  std::copy(out, out + nq, p->q);
  std::copy(out + nq, out + nq + nt, p->t);
  const double* X = out + nq + nt;
  for (int i = 0; i < P_; ++i) {
    const int pt = point_perm_[i];
    for (int a = 0; a < 4; ++a) p->X[4 * pt + a] = X[4 * i + a];
  }
  if (nk) std::copy(out + nq + nt + nx, out + tot, p->k);
}

void BaSolver::Solve(const sg_solver_options& o, sg_problem* p, sg_solver_summary* s) {
  Begin(o);
  const int batch = 8;
  LmState h{};
  const long long cap = (long long)o.max_num_iterations * (o.max_num_consecutive_invalid_steps + 2) + 16;
  long long launched = 0;
  while (true) {
    Iterate(batch);
    launched += batch;
    ReadState(&h);
    if (h.done) break;
    SG_REQUIRE(launched < cap, SG_EDEVICE, "LM loop did not terminate on the device");
  }
  Summary(s);
  Download(p);
}

void BaSolver::Evaluate(double* residuals, double* cost, int32_t* nfail) {
  SG_REQUIRE(loaded_, SG_EINVAL, "no problem loaded");
  DBuf<double> r, c;
  DBuf<int32_t> nf;
  r.Resize(2 * (size_t)std::max(M_, 1));
  c.Resize(1);
  nf.Resize(1);
  c.Zero(stream_);
  nf.Zero(stream_);
  Dev d = MakeDev();
  if (M_ > 0)
    LaunchEvaluateK(M_, stream_, d, r.ptr, c.ptr, nf.ptr);
  std::vector<double> rh(2 * (size_t)M_);
  if (M_ > 0) SG_HIP_CHECK(hipMemcpyAsync(rh.data(), r.ptr, rh.size() * 8, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipMemcpyAsync(cost, c.ptr, 8, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipMemcpyAsync(nfail, nf.ptr, 4, hipMemcpyDeviceToHost, stream_));
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
  for (int o = 0; o < M_; ++o) {
    residuals[2 * obs_perm_[o]] = rh[2 * o];
    residuals[2 * obs_perm_[o] + 1] = rh[2 * o + 1];
  }
}

void BaSolver::SetTiming(bool on) {
  timing_ = on;
  for (auto& t : timers_) {
    for (auto e : t.ev) (void)hipEventDestroy(e);
    t.ev.clear();
    t.total_ms = 0.0;
    t.count = 0;
  }
}

void BaSolver::CollectTimes() {
  SG_HIP_CHECK(hipStreamSynchronize(stream_));
  for (auto& t : timers_) {
    for (size_t i = 0; i + 1 < t.ev.size(); i += 2) {
      float ms = 0.f;
      SG_HIP_CHECK(hipEventElapsedTime(&ms, t.ev[i], t.ev[i + 1]));
      t.total_ms += ms;
      t.count += 1;
    }
    for (auto e : t.ev) (void)hipEventDestroy(e);
    t.ev.clear();
  }
}

int BaSolver::KernelTimes(char* names, int names_len, double* ms, int32_t* counts, int max) {
  CollectTimes();
  std::string all;
  int k = 0;
  for (auto& t : timers_) {
    if (k < max) {
      ms[k] = t.count ? t.total_ms / t.count : 0.0;
      counts[k] = t.count;
    }
    if (!all.empty()) all += ",";
    all += t.name;
    ++k;
  }
  if (names && names_len > 0) {
    std::strncpy(names, all.c_str(), names_len - 1);
    names[names_len - 1] = 0;
  }
  return std::min(k, max);
}

// Algorithmic bytes / flops per launch (for the roofline line in bench.py).
int BaSolver::KernelWork(double* bytes, double* flops, int max) {
  const double M = M_, P = P_, n = n_, NB = NB_;
  double npairs = 0.0;  // observation pairs of free points on free frames are not tracked here: use M*k/2
  (void)npairs;
  std::vector<double> by(kKNum, 0.0), fl(kKNum, 0.0);
  // linearize: read obs (16 B pt + 4 B frame + 1 B fixed) + point X 32 B + offsets 4 B; write the J record
  // (kJStride doubles: 128 B since round 6), V 80 B, g 32 B per point; camera partials
  const double jrec = 8.0 * kJStride;
  by[kKLin] = M * (16 + 4 + 1 + jrec) + P * (32 + 4 + 80 + 32 + 1) + NB * kCamV * 8;
  fl[kKLin] = M * 420.0;
  // k_schur: the record less r~ (rotation pairs + J~p) and the observation meta; per point V, g, scales, X.w and
  // the written Vinv / t / diag
  by[kKSchur] = M * (jrec - 16 + 4) + P * (80 + 32 + 32 + 8 + 32 + 80 + 32);
  fl[kKSchur] = 2048.0 * schur_mfma_ + 512.0 * schur_rhs_;   // 16x16x4 tile updates, 4x4x4 (4-block) rhs slots
  by[kKPointUpd] = M * (jrec + 16 + 4) + P * (32 + 32 + 80 + 32 + 32);
  if (spec_) {   // k_update_lin: the update's traffic plus the candidate's linearization (a second J record, V, g)
    by[kKPointUpd] = M * (jrec + jrec + 16 + 4 + 4 + 4) + P * (32 + 32 + 80 + 32 + 32 + 80 + 32) + NB * kCamV * 8;
    fl[kKPointUpd] = M * 420.0;
  }
  by[kKChol] = n * n * 8 * 2;
  fl[kKChol] = n * n * n / 3.0;
  int k = 0;
  for (; k < std::min(max, (int)kKNum); ++k) {
    bytes[k] = by[k];
    flops[k] = fl[k];
  }
  // derived figures after the kernels (bench.py's roofline fields):
  //   [kKNum]     k_schur's useful flops: the MFMA slots of each point's own tiles (its first to its last window
  //               tile), without the slots that multiply the zero tiles left of its first column
  //   [kKNum + 1] SURVEY 8d's algorithmic bytes of one linearization sweep at the reference's f64: per observation
  //               uv 16 + frame index 4 + r 16 + W_ip 192, per point CSR offset 4 + X 32 + V_p 80 + g_p 32, per
  //               camera block pose 56 + U_i / g_c 8 (21 + 6)
  if (max > kKNum) {
    bytes[kKNum] = 0.0;
    flops[kKNum] = schur_useful_;
    ++k;
  }
  if (max > kKNum + 1) {
    bytes[kKNum + 1] = M * 228.0 + P * 148.0 + NB * (56.0 + 8.0 * 27);
    flops[kKNum + 1] = 0.0;
    ++k;
  }
  return k;
}

void BaSolver::Info(sg_ba_info* o) const {
  std::memset(o, 0, sizeof(*o));
  o->num_frames = F_;
  o->num_points = P_;
  o->num_obs = M_;
  o->num_blocks = NB_;
  o->n = n_;
  o->band_tiles = band_tiles_;
  o->cholesky_path = chol_border_ ? 4 : chol_tiles_ ? 0 : (chol_window_ ? 1 : (chol_gstage_ ? 2 : 3));
  o->cholesky_split = chol_tiles_ ? chol_nd_ : 0;
  o->num_pairs = (int32_t)std::min<size_t>(npairs_, INT32_MAX);
  o->rank = comm_ ? comm_->rank() : 0;
  o->nranks = comm_ ? comm_->nranks() : 1;
  o->num_allreduces = nallreduce_;
  o->lin_waves = lin_waves_;
  o->cholesky_separator = chol_tiles_ && chol_nd_ > 0 ? chol_ns_ : 0;
}

double BaSolver::ReprojectMap(sg_map* m) {
  SG_HIP_CHECK(hipSetDevice(dev_.device));
  const int M = m->num_obs;
  hipStream_t s = stream_;
  io_.Begin();
  io_.Up(mk_, m->k, 7 * (size_t)m->num_cameras);
  io_.Up(mq_, m->q, 4 * (size_t)m->num_frames);
  io_.Up(mt_, m->t, 3 * (size_t)m->num_frames);
  io_.Up(mX_, m->X, 4 * (size_t)m->num_points);
  io_.Up(mobs_pt_, m->obs_pt, 2 * (size_t)M);
  io_.Up(mobs_frame_, m->obs_frame, (size_t)M);
  io_.Up(mobs_point_, m->obs_point, (size_t)M);
  io_.Up(mframe_cam_, m->frame_camera, (size_t)m->num_frames);
  io_.FlushUp(s);
  mobs_err_.Resize(2 * (size_t)std::max(M, 1));
  const int nb = std::max((M + 255) / 256, 1);
  mred_.Resize(2 * (size_t)nb + 2);   // (every block writes its partial: no zeroing)
  LaunchReprojectMapK(M, nb, s, mk_.ptr, mq_.ptr, mt_.ptr, mframe_cam_.ptr, mX_.ptr, mobs_pt_.ptr, mobs_frame_.ptr,
                      mobs_point_.ptr, mobs_err_.ptr, mred_.ptr);
  SG_HIP_CHECK(hipGetLastError());
  double out[2] = {0, 0};
  io_.Down(m->obs_error, mobs_err_.ptr, 2 * (size_t)M * 8);
  io_.Down(out, mred_.ptr + 2 * nb, 16);
  io_.FinishDown(s);
  return out[0];
}

}  // namespace sg
