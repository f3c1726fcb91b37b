/*
 * slamgpu.h — C-ABI of the MI355X-native local-mapping back end (libslamgpu.so).
 *
 * The drop-in boundary for the reference's hot path (ywrt/slam-robot):
 *   - class Slam            (slam.h:21-65)  -> sg_slam_* (SolveFrames / SolveAllFrames / ReprojectMap,
 *                                              iterations(), error())
 *   - Ceres problem + solve (slam.cpp:257-521) -> sg_problem_* / sg_ba_*  (compact problem, LM solve)
 *   - ProjectPoint          (project.h:11-54) -> device code inside the solver and sg_project_points
 *   - HessianTracker        (hessian.h:9-270) -> sg_tracker_*           (front end, see sg_track_*)
 *
 * Conventions: plain pointers and sizes only, no C++/torch types.  Every entry point returns 0 (SG_OK) on
 * success or a negative errno-style code.  The caller owns every host array it passes; the library owns
 * its device buffers (allocated on first use, grown on demand, freed by *_destroy).  One handle per host
 * thread; each handle owns one HIP stream on the device named in its options.
 */
#ifndef SLAMGPU_H_
#define SLAMGPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_OK 0
#define SG_EINVAL (-22)   /* bad argument / inconsistent sizes */
#define SG_ENOMEM (-12)   /* host or device allocation failed */
#define SG_EDEVICE (-5)   /* HIP runtime error (message via sg_last_error) */
#define SG_ENODEV (-19)   /* no usable gfx950 device */
#define SG_ECOMM (-71)    /* RCCL error */

/* Bit positions of TrackedPoint::Flags (localmap.h:184-190). point_flags holds (1 << flag). */
enum sg_point_flag {
  SG_BAD_LOCATION = 0,
  SG_NO_BASELINE = 1,
  SG_NO_OBSERVATIONS = 2,
  SG_MISMATCHED = 3,
  SG_BAD_FEATURE = 4
};

/* Termination types (ceres::SolverTerminationType, Ceres 1.8 naming). */
enum sg_termination {
  SG_NO_CONVERGENCE = 0,
  SG_FUNCTION_TOLERANCE = 1,
  SG_GRADIENT_TOLERANCE = 2,
  SG_PARAMETER_TOLERANCE = 3,
  SG_NUMERICAL_FAILURE = 4,
  SG_DID_NOT_RUN = 5,
  SG_DEVICE_TIMEOUT = 6   /* not a Ceres type: a device hand-off of the Cholesky hit its spin limit (the GPU was
                             shared or stalled); the step is not trusted and the solve fails (ok = 0) */
};

/*
 * LocalMap (localmap.h:284-320) in structure-of-arrays form.  Frames are in LocalMap::frames order,
 * observations grouped by frame in Frame::observations() order.  q/t/X/k are the parameter blocks the
 * reference hands to Ceres by raw pointer (localmap.h:129-132,159-160,194-195,30); they are updated in
 * place by a solve exactly as Ceres updates the map's own storage.
 */
typedef struct sg_map {
  int32_t num_cameras;
  double* k;                    /* [7*num_cameras]  Camera::k = k1,k2,k3,fx,fy,cx,cy */
  int32_t num_frames;
  double* q;                    /* [4*F] Frame::rotation().coeffs()  Eigen order [x,y,z,w] */
  double* t;                    /* [3*F] Frame::translation() */
  const int32_t* frame_camera;  /* [F] index into cameras */
  const int32_t* frame_prev;    /* [F] index of Frame::previous(), -1 if none */
  int32_t num_points;
  double* X;                    /* [4*P] TrackedPoint::location() homogeneous [X,Y,Z,W] */
  int32_t* point_flags;         /* [P] TrackedPoint flags bitmask */
  double* point_uncertainty;    /* [P] TrackedPoint::uncertainty() */
  int32_t num_obs;
  const double* obs_pt;         /* [2*M] Observation::pt (pixels) */
  const int32_t* obs_frame;     /* [M] */
  const int32_t* obs_point;     /* [M] */
  int32_t* obs_disabled;        /* [M] Observation::is_disabled */
  double* obs_error;            /* [2*M] Observation::error, written by ReprojectMap */
} sg_map;

/*
 * The Ceres problem that Slam::SetupProblem builds (slam.cpp:257-414), in compact form.
 *   - one quaternion block (4, local 3 via ceres::QuaternionParameterization) + one translation block (3)
 *     per frame; a frame's blocks are free or constant independently (the translation of a skipped
 *     previous frame can be free through FrameDistance while its rotation is absent);
 *   - one homogeneous point block (4, no parameterization) per point, free or constant;
 *   - intrinsics blocks (7) per camera, constant unless cameras_free (SolveAllFrames(..., true));
 *   - residual blocks: ReprojectionError (2) with CauchyLoss(range) per observation, FrameDistance (1)
 *     with CauchyLoss(dist_range) per (frame, prev) pair, CameraStabilization (7) with CauchyLoss(5)
 *     per camera when cameras_free.
 */
typedef struct sg_problem {
  int32_t num_cameras;
  double* k;                    /* [7*ncam] */
  int32_t cameras_free;         /* 0: intrinsics constant (SolveFrames) */
  int32_t num_frames;
  double* q;                    /* [4*F] updated in place */
  double* t;                    /* [3*F] updated in place */
  int32_t* frame_camera;        /* [F] */
  uint8_t* frame_rot_free;      /* [F] */
  uint8_t* frame_trans_free;    /* [F] */
  int32_t* frame_map_index;     /* [F] source frame in the sg_map, or -1 */
  int32_t num_points;
  double* X;                    /* [4*P] updated in place */
  uint8_t* point_free;          /* [P] */
  int32_t* point_map_index;     /* [P] source point in the sg_map, or -1 */
  int32_t num_obs;
  double* obs_pt;               /* [2*M] observed pixel */
  int32_t* obs_frame;           /* [M] problem frame index */
  int32_t* obs_point;           /* [M] problem point index */
  int32_t num_dist;
  int32_t* dist_frame;          /* [D] FrameDistance(frame.t, prev.t) */
  int32_t* dist_prev;           /* [D] */
  double range;                 /* CauchyLoss(range) on reprojection (slam.cpp:265) */
  double dist_target;           /* FrameDistance(150.) (slam.cpp:403) */
  double dist_range;            /* CauchyLoss(15) (slam.cpp:404) */
  double stab_range;            /* CauchyLoss(5) on CameraStabilization (slam.cpp:463) */
  void* owner_;                 /* library-owned storage (sg_problem_from_map), NULL for caller-owned */
} sg_problem;

/* ceres::Solver::Options as used by Slam::Run (slam.cpp:482-508) plus the Ceres 1.8 defaults it keeps. */
typedef struct sg_solver_options {
  int32_t max_num_iterations;            /* 1000 (slam.cpp:493) */
  double function_tolerance;             /* 1e-7 (slam.cpp:494); 1e-9 when fine */
  double gradient_tolerance;             /* 1e-10, relative to the initial gradient max-norm (Ceres 1.8) */
  double parameter_tolerance;            /* 1e-8 */
  double min_relative_decrease;          /* 1e-3 */
  double initial_trust_region_radius;    /* 1e4 */
  double max_trust_region_radius;        /* 1e16 */
  double min_trust_region_radius;        /* 1e-32 */
  double min_lm_diagonal;                /* 1e-6 */
  double max_lm_diagonal;                /* 1e32 */
  int32_t max_num_consecutive_invalid_steps; /* 5 */
  int32_t jacobi_scaling;                /* 1 */
  int32_t disable_termination;           /* benchmark mode: run exactly max_num_iterations LM iterations */
  int32_t always_linearize;              /* benchmark mode: a rejected step re-linearizes too (same values),
                                            so every iteration is SURVEY.md 8d's full unit of work; 0 = Ceres */
} sg_solver_options;

/* ceres::Solver::Summary fields the reference reads (slam.cpp:510-520). */
typedef struct sg_solver_summary {
  int32_t num_iterations;        /* summary.iterations.size() — includes iteration 0 (slam.cpp:517) */
  int32_t num_successful_steps;
  int32_t num_unsuccessful_steps;
  int32_t num_invalid_steps;
  int32_t termination_type;      /* enum sg_termination */
  int32_t ok;                    /* summary.error.empty() (slam.cpp:520) */
  double initial_cost;           /* including fixed cost */
  double final_cost;             /* summary.final_cost (slam.cpp:518) */
  double fixed_cost;
  double trust_region_radius;
  int32_t num_lm_iterations;     /* LM loop iterations executed on the device (benchmark unit) */
  int32_t sync_timeouts;         /* Cholesky hand-off waits that hit their spin limit (0 in a healthy solve; a
                                    non-zero count ends the solve with SG_DEVICE_TIMEOUT) */
} sg_solver_summary;

typedef struct sg_device_options {
  int32_t device;                /* HIP device ordinal */
  int32_t precision;             /* 0: fp64 everywhere, the reference's arithmetic (the only mode: any other
                                    value is rejected with SG_EINVAL) */
  int32_t rank;                  /* landmark shard index (0 for single GPU) */
  int32_t nranks;                /* 1 for single GPU */
} sg_device_options;

/* ---------------------------------------------------------------------------------------------------- */
/* Library */
const char* sg_version(void);
const char* sg_last_error(void);              /* thread-local message for the last failing call */
void sg_solver_options_default(sg_solver_options* o);
void sg_device_options_default(sg_device_options* o);

/* ---------------------------------------------------------------------------------------------------- */
/* Problem assembly (host side of Slam::SetupProblem, slam.cpp:257-414 / SolveFrames 417-443 /
 * SolveAllFrames 447-480).  Returns 1 in *built when the problem was built, 0 when the reference aborts
 * ("Slam aborted due to frame set too small", slam.cpp:305-308). */
int sg_problem_from_map_frames(const sg_map* map, int32_t num_to_solve, int32_t num_to_present,
                               double range, sg_problem* out, int32_t* built);
int sg_problem_from_map_all(const sg_map* map, double range, int32_t solve_cameras,
                            sg_problem* out, int32_t* built);
void sg_problem_free(sg_problem* p);
/* Copy solved parameter blocks back into the map (what Ceres does through the raw pointers). */
int sg_problem_write_back(const sg_problem* p, sg_map* map);
/* Split a problem's landmarks into nranks shards (contiguous ranges of points sorted by first observing
 * frame); every shard keeps all frames, cameras and FrameDistance blocks. */
int sg_problem_shard(const sg_problem* p, int32_t rank, int32_t nranks, sg_problem* out);

/* ---------------------------------------------------------------------------------------------------- */
/* Device bundle-adjustment solver (Ceres 1.8 Levenberg-Marquardt + SPARSE_SCHUR, restated on MI355X). */
typedef struct sg_ba sg_ba;
int sg_ba_create(sg_ba** out, const sg_device_options* dev);
void sg_ba_destroy(sg_ba* h);
/* RCCL communicator for landmark sharding: id is ncclUniqueId (128 bytes), from sg_comm_unique_id. */
int sg_comm_unique_id(void* id128);
int sg_ba_comm_init(sg_ba* h, const void* id128, int32_t nranks, int32_t rank);
/* In-process communicator group: nranks (<= 8) solver handles on ONE device, each driven by its own host
 * thread, exchange through the group instead of RCCL (each all-reduce synchronises the rank's stream, meets
 * the others at a host barrier and sums in rank order).  Runs the landmark-sharded device chain (envelope
 * union, rank-0 assembly, packed S exchange, the replicated decision) on a one-GPU machine; for tests.
 * Destroy the group after every handle that uses it. */
typedef struct sg_comm_group sg_comm_group;
int sg_comm_group_create(sg_comm_group** out, int32_t nranks);
void sg_comm_group_destroy(sg_comm_group* g);
int sg_ba_comm_init_local(sg_ba* h, sg_comm_group* g, int32_t rank);
/* Host-callback communicator: one process per rank over any host collective (gloo, MPI).  Each of the solver's
 * all-reduces copies its device buffer to host memory, calls fn(buf, n, op, user) (op 0 = sum, 1 = max; return
 * 0 on success, nonzero fails the call with SG_ECOMM) and copies the result back — the call sequence of the
 * RCCL communicator (sg_ba_comm_init), with the transport on the host.  Must precede sg_ba_load. */
typedef int (*sg_allreduce_fn)(double* buf, long long n, int32_t op, void* user);
int sg_ba_comm_init_host(sg_ba* h, int32_t nranks, int32_t rank, sg_allreduce_fn fn, void* user);
/* Upload a problem (the problem's q/t/X are read now and written back by sg_ba_download). */
int sg_ba_load(sg_ba* h, const sg_problem* p);
/* Pre-size the handle's device and pinned staging buffers for problems of up to max_frames frames, max_points
 * points and max_obs observations (a map's high-water mark), so loads that follow do not reallocate on their
 * critical path.  Reallocation drops the loaded problem (load again).  The Slam facade does this itself,
 * reserving twice the largest window problem it has loaded. */
int sg_ba_reserve(sg_ba* h, int32_t max_frames, int32_t max_points, int32_t max_obs);
/* Incremental problem update (replaces the per-call rebuild of slam.cpp:257-414): a
 * load whose structure equals the previous load's (frames, cameras, freedom flags, observation incidence,
 * FrameDistance pairs) re-uploads the values only.  Counts of full and value-only loads on this handle. */
int sg_ba_load_counts(const sg_ba* h, int32_t* full_loads, int32_t* value_loads);
/* Run the LM solve on the device; writes the solved blocks back into p. */
int sg_ba_solve(sg_ba* h, const sg_solver_options* o, sg_problem* p, sg_solver_summary* s);
/* Benchmark entry: (re)initialise from the uploaded state, then enqueue exactly n LM iterations without
 * host synchronisation (termination disabled).  sg_ba_sync waits for completion. */
int sg_ba_begin(sg_ba* h, const sg_solver_options* o);
int sg_ba_iterate(sg_ba* h, int32_t n);
int sg_ba_sync(sg_ba* h);
int sg_ba_summary(sg_ba* h, sg_solver_summary* s);
int sg_ba_download(sg_ba* h, sg_problem* p);
/* Per-kernel timing over the last sg_ba_iterate calls (HIP events on the solver's stream). names is a
 * comma-separated list; ms[i] = mean duration of kernel i per launch; counts[i] launches timed. */
int sg_ba_set_timing(sg_ba* h, int32_t enable);
int sg_ba_kernel_times(sg_ba* h, char* names, int32_t names_len, double* ms, int32_t* counts, int32_t max);
/* Algorithmic byte / flop counts for the roofline (per launch of each timed kernel). */
int sg_ba_kernel_work(sg_ba* h, double* bytes, double* flops, int32_t max);

/* What the last sg_ba_load set up (diagnostics, benchmark records, shard balance). */
typedef struct sg_ba_info {
  int32_t num_frames, num_points, num_obs;   /* the loaded problem (this rank's landmark shard) */
  int32_t num_blocks;                        /* free camera blocks (frames with a free rotation or translation) */
  int32_t n;                                 /* reduced camera system dimension (6 blocks + free intrinsics) */
  int32_t band_tiles;                        /* widest row of the Cholesky envelope, in 16-wide tiles */
  int32_t cholesky_path;                     /* 0: tiled band (k_chol_tiles), 1: LDS window, 2: global memory
                                                (panel rows staged in LDS), 3: global memory, 4: bordered band
                                                (free intrinsics: frame band tiled, then the border) */
  int32_t num_pairs;                         /* Schur observation pairs (s <= t) of this rank's free points */
  int32_t rank, nranks;
  int32_t cholesky_split;                    /* tiled path: tile rows factored bottom-up by a second workgroup
                                                (dissected band; 0: one workgroup) */
  int32_t num_allreduces;                    /* landmark-shard sum all-reduces this handle has issued in LM
                                                iterations (0 on one rank) */
  int32_t lin_waves;                         /* waves per Jacobian-sweep chunk (1, or 2 when the doubled grid
                                                fits the device at once) */
  int32_t cholesky_separator;                /* tiled path with a split: the separator's tile rows (<= 7) */
} sg_ba_info;
int sg_ba_info_get(const sg_ba* h, sg_ba_info* out);

/* Jacobian/Hessian sweep only (benchmark of the HBM-bound kernel): n linearizations at the current
 * state (k_linearize + camera-block reduce), timed when sg_ba_set_timing is on. */
int sg_ba_sweep(sg_ba* h, int32_t n);

/* Residual sweep only (ReprojectionError over the uploaded observations at the current state):
 * r[2*M] corrected residuals in problem order, returns cost (without fixed cost) and failure count. */
int sg_ba_evaluate(sg_ba* h, double* residuals, double* cost, int32_t* num_failed);

/* ---------------------------------------------------------------------------------------------------- */
/* Slam facade (slam.h:21-65).  A handle keeps iterations()/error() like the reference's Slam object. */
typedef struct sg_slam sg_slam;
int sg_slam_create(sg_slam** out, const sg_device_options* dev);
void sg_slam_destroy(sg_slam* s);
int sg_slam_solve_frames(sg_slam* s, sg_map* map, int32_t num_to_solve, int32_t num_to_present,
                         double range, int32_t* solved);                          /* slam.cpp:417-443 */
int sg_slam_solve_all_frames(sg_slam* s, sg_map* map, double range, int32_t solve_cameras,
                             int32_t* solved);                                    /* slam.cpp:447-480 */
int sg_slam_reproject_map(sg_slam* s, sg_map* map, double* mean);               /* slam.cpp:523-548 */
int32_t sg_slam_iterations(const sg_slam* s);                                    /* slam.h:49 */
double sg_slam_error(const sg_slam* s);                                          /* slam.h:50 */
int sg_slam_load_counts(const sg_slam* s, int32_t* full_loads, int32_t* value_loads);   /* see sg_ba_load_counts */
/* Host wall time (ms) of the last SolveFrames / SolveAllFrames call by phase: [0] SetupProblem (problem build),
 * [1] sg_ba_load (work lists + upload), [2] device LM loop incl. download, [3] write-back into the map.
 * A development aid for sizing the host share of a real call (tools/e2e_replay.py). */
int sg_slam_last_phase_ms(const sg_slam* s, double* ms4);
int sg_slam_last_summary(const sg_slam* s, sg_solver_summary* out);

/* ------------------------------------------------------------------------------------------------
 * Front end: HessianTracker (hessian.h:9-270) and the forward/backward matching step of Matcher
 * (matcher.cpp:173-206 TrackFeature, 247-251 the 3 -> 6 level retry).  A tracker holds `max_images`
 * device pyramids ("views", matcher.cpp:36-40); images are 8-bit, 3 channels, cv::Mat (BGR) memory order.
 */
typedef struct sg_tracker sg_tracker;

typedef struct sg_tracker_options {
  int32_t window;          /* patch size W: kWindowSize = 13 (matcher.cpp:27); 1..16 */
  int32_t depth;           /* pyramid levels per image: MakePyramid(img, 6) (matcher.cpp:221); 1..8 */
  int32_t max_iterations;  /* Track() Newton iterations: 10 (matcher.cpp:176) */
  float threshold;         /* Track() convergence threshold: 0.001 (matcher.cpp:176) */
  float fb_max;            /* forward/backward disagreement limit: 0.3 px (matcher.cpp:200) */
  int32_t retry_levels;    /* levels of the retry after a failed attempt: 6 (matcher.cpp:248); 0 = none */
  int32_t max_images;      /* pyramid slots held on the device */
  int32_t mode;            /* FeatureTracker implementation: SG_TRACKER_HESSIAN (the one Matcher uses,
                              matcher.cpp:20), SG_TRACKER_KLT (klt.h), SG_TRACKER_BRUTE (brute.h) */
  int32_t reserved[4];
} sg_tracker_options;

enum sg_tracker_mode { SG_TRACKER_HESSIAN = 0, SG_TRACKER_KLT = 1, SG_TRACKER_BRUTE = 2 };

void sg_tracker_options_default(sg_tracker_options* o);
int sg_tracker_create(sg_tracker** out, const sg_tracker_options* o, const sg_device_options* dev);
void sg_tracker_destroy(sg_tracker* t);

/* MakePyramid (hessian.h:95-126) of one image into pyramid slot `slot`. */
int sg_tracker_set_image(sg_tracker* t, int32_t slot, const uint8_t* bgr, int32_t width, int32_t height,
                         int32_t stride);
/* Download pyramid level `level` of slot `slot` (width*height floats). */
int sg_tracker_get_level(sg_tracker* t, int32_t slot, int32_t level, float* out, int32_t* width,
                         int32_t* height);
/* GetPatch (hessian.h:54-93) at n points of one level: out[n][W*W], mean[n], sumsq[n]. */
int sg_tracker_get_patches(sg_tracker* t, int32_t slot, int32_t level, int32_t n, const float* xy, float* out,
                           float* mean, float* sumsq);
/* Forward/backward tracking of n features from slot `from` to slot `to` (synchronous).  levels[i] is 3 or 6
 * (matcher.cpp:234-236); to_xy: in = starting guess, out = the matcher's to_pt; accepted[i] = 1 if the
 * feature matched; iterations (may be NULL) = Newton iterations spent per feature. */
int sg_tracker_track(sg_tracker* t, int32_t from, int32_t to, int32_t n, const float* from_xy, float* to_xy,
                     const int32_t* levels, int32_t* accepted, int32_t* iterations);
/* Device-resident variant for throughput runs: load features once, run `repeats` asynchronous tracking
 * passes (each restarts from the loaded starting guesses), then fetch the last pass's results. */
/* One-directional TrackFeature of the tracker's mode for n features (hessian.h:243-264, klt.h:403-424,
 * brute.h:129-164): templates GetPatches(from slot, from_xy) (levels[i] of them in HESSIAN mode, NULL = all;
 * every level in the other modes), then coarse-to-fine tracking in the `to` slot starting from to_xy, with
 * threshold / max_iterations from the options.  to_xy is updated only where status is 0 (OK); 2 =
 * OUT_OF_BOUNDS.  iterations (optional): Newton iterations run (0 in BRUTE mode). */
int sg_tracker_track_feature(sg_tracker* t, int32_t from, int32_t to, int32_t n, const float* from_xy, float* to_xy,
                             const int32_t* levels, int32_t* status, int32_t* iterations);
int sg_tracker_load_features(sg_tracker* t, int32_t n, const float* from_xy, const float* to_xy,
                             const int32_t* levels);
int sg_tracker_run(sg_tracker* t, int32_t from, int32_t to, int32_t repeats);
int sg_tracker_results(sg_tracker* t, float* to_xy, int32_t* accepted, int32_t* iterations);
/* New-keyframe corner seeding of Matcher::Track (matcher.cpp:123-169, 214, 380-383) on the image of `slot`:
 * grey = cvtColor(BGR, CV_RGB2GRAY); goodFeaturesToTrack(grey, max_corners = 120, quality = 0.01,
 * min_distance = 20) (Shi-Tomasi, blockSize 3, strongest first, ties in row-major order); then
 * AddNewFeatures' 30 x 30 grid: a corner is added unless its cell is within one cell of a match.
 * corners_xy / added_xy hold up to max_corners points each (x, y). */
int sg_tracker_seed_features(sg_tracker* t, int32_t slot, const float* match_xy, int32_t num_matches,
                             int32_t max_corners, double quality, double min_distance, float* corners_xy,
                             int32_t* num_corners, float* added_xy, int32_t* num_added);
/* Kernel timing (HIP events on the tracker's stream) of the last sg_tracker_run: total ms of the
 * tracking kernels and of the pyramid kernels of the last sg_tracker_set_image. */
int sg_tracker_kernel_ms(sg_tracker* t, double* track_ms, double* pyramid_ms);

/* ------------------------------------------------------------------------------------------------
 * All-pairs 256-bit descriptor matching (the matcher's brute-force descriptor distance; BASELINE config 4).
 * Descriptors are 4 x uint64 per row.  Per query row: best_idx = argmin over train rows of
 * popcount(q XOR t) with ties to the lowest index, best_dist, and second_dist = the second-smallest
 * distance (equal to best_dist on a tie); -1 where the train set is too small.
 */
typedef struct sg_matcher sg_matcher;
int sg_matcher_create(sg_matcher** out, const sg_device_options* dev);
void sg_matcher_destroy(sg_matcher* m);
int sg_hamming_match(sg_matcher* m, const uint64_t* query, int32_t nq, const uint64_t* train, int32_t nt,
                     int32_t* best_idx, int32_t* best_dist, int32_t* second_dist);
/* Device-resident throughput path: load once, run `repeats` asynchronous passes, fetch results and the
 * average kernel time per pass (HIP events). */
int sg_hamming_load(sg_matcher* m, const uint64_t* query, int32_t nq, const uint64_t* train, int32_t nt);
int sg_hamming_run(sg_matcher* m, int32_t repeats);
int sg_hamming_results(sg_matcher* m, int32_t* best_idx, int32_t* best_dist, int32_t* second_dist,
                       double* kernel_ms);
int sg_slam_set_options(sg_slam* s, const sg_solver_options* o);

/* LocalMap maintenance on the device, run on the residuals sg_slam_reproject_map wrote (main.cpp:584-599).
 * A point's observation order (TrackedPoint::observations()) is ascending frame index, ties by map index
 * (Frame::Commit, localmap.cpp:85-89). */
/* LocalMap::Clean(error_threshold) (localmap.cpp:283-398): fixes X[4p+3], writes point_flags,
 * point_uncertainty and obs_disabled; *result = the reference's bool (0 when observations were disabled). */
int sg_map_clean(sg_slam* s, sg_map* map, double error_threshold, int32_t* result);
/* LocalMap::ApplyEpipolarConstraint() (localmap.cpp:232-276): writes point_flags and obs_disabled;
 * *num_violations = points whose |h2^T E h1| exceeded 0.15. */
int sg_map_apply_epipolar(sg_slam* s, sg_map* map, int32_t* num_violations);
/* LocalMap::Normalize (localmap.cpp:114-155): translate frame 0 to the origin, then rotate frame 0 to the
 * identity (frames' rotations and translations, points' homogeneous locations; a map with < 2 frames is left
 * alone).  main.cpp:602-605 checks that ReprojectMap is unchanged by it (CHECK_NEAR 0.1). */
int sg_map_normalize(sg_slam* s, sg_map* map);

/* ------------------------------------------------------------------------------------------------
 * Matcher::Track (matcher.h:20-26, matcher.cpp:301-405): the per-frame front end with its bookkeeping —
 * live features (ordered by TrackedPoint id), up to four keyframe views whose pyramids stay resident on the
 * device, FindMatches (matcher.cpp:210-271) batched over features on the device, the keyframe decision
 * (< 40 matches), corner seeding of new points (AddNewFeatures + Unproject at 2000) and view expiry.
 * The LocalMap stays the caller's: the library reads and grows it through these callbacks, which stand in
 * for the reference's direct member access (each cites what it replaces).  Callbacks return 0 on success;
 * a non-zero return aborts the call with SG_EINVAL.
 */
typedef struct sg_map_callbacks {
  void* user;
  /* Frame::rotation().coeffs() [x,y,z,w], translation(), camera()->k (localmap.h:129-132,159-160,30) */
  int32_t (*frame_pose)(void* user, int32_t frame, double* q4, double* t3, double* k7);
  /* TrackedPoint::location(), uncertainty(), feature_usable() (localmap.h:194-195,251,249) */
  int32_t (*point_state)(void* user, int32_t point, double* X4, double* uncertainty, int32_t* feature_usable);
  /* LocalMap::AddPoint(id, location) (localmap.cpp:103-109): NO_OBSERVATIONS | NO_BASELINE flags,
   * uncertainty 1e8.  Writes the new point's handle to *point. */
  int32_t (*add_point)(void* user, int32_t id, const double* X4, int32_t* point);
  /* Frame::AddObservation(pt, point) (localmap.h:138-143) */
  int32_t (*add_observation)(void* user, int32_t frame, double x, double y, int32_t point);
  /* frame->is_keyframe_ = true (matcher.cpp:357) */
  int32_t (*set_keyframe)(void* user, int32_t frame);
  /* Matcher::Track's update_frames argument (may be NULL): *updated = its bool result */
  int32_t (*update_frames)(void* user, int32_t* updated);
} sg_map_callbacks;

typedef struct sg_frontend_stats {
  int32_t matches_first;   /* "Started with %d" (matcher.cpp:341) */
  int32_t matches;         /* "grew to %d" */
  int32_t keyframe;        /* 1 when the frame became a keyframe */
  int32_t corners;         /* goodFeaturesToTrack corners on a keyframe */
  int32_t added;           /* new features / points ("Added %d new features") */
  int32_t features;        /* live features after the call */
  int32_t views;           /* keyframe views after the call */
  int32_t track_batches;   /* device FindMatches launches (one per pass; a second after update_frames) */
} sg_frontend_stats;

typedef struct sg_frontend sg_frontend;
/* o: tracker options (window 13, depth 6 for the reference's Matcher; NULL = defaults). */
int sg_frontend_create(sg_frontend** out, const sg_tracker_options* o, const sg_device_options* dev);
void sg_frontend_destroy(sg_frontend* f);
/* Matcher::Track(img, frame, camera, map, update_frames): *result = the reference's bool (always 1). */
int sg_frontend_track(sg_frontend* f, const uint8_t* bgr, int32_t width, int32_t height, int32_t stride,
                      int32_t frame, int32_t camera, const sg_map_callbacks* cb, int32_t* result,
                      sg_frontend_stats* stats);
/* Live features: point handles and TrackedPoint ids in set order (ids ascending); n in/out = capacity/count. */
int sg_frontend_features(sg_frontend* f, int32_t* points, int32_t* ids, int32_t* n);

#ifdef __cplusplus
}
#endif
#endif /* SLAMGPU_H_ */
