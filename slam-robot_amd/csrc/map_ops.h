// map_ops.h — LocalMap maintenance on the device (Clean, ApplyEpipolarConstraint, Normalize); see map_ops.hip.
#ifndef SG_MAP_OPS_H_
#define SG_MAP_OPS_H_

#include <hip/hip_runtime.h>

#include "common.h"
#include "dbuf.h"
#include "hostio.h"

namespace sg {

class MapOps {
 public:
  // stream: the HIP stream to run on (the Slam facade passes its solver's, so the object uses one hardware
  // queue); nullptr: a stream of its own
  explicit MapOps(const sg_device_options& dev, hipStream_t stream = nullptr);
  ~MapOps();
  // LocalMap::Clean (localmap.cpp:283-398): returns the reference's bool (0 when observations were disabled).
  int Clean(sg_map* m, double error_threshold);
  // LocalMap::ApplyEpipolarConstraint (localmap.cpp:232-276): returns the number of points over the cut.
  int ApplyEpipolarConstraint(sg_map* m);
  // LocalMap::Normalize (localmap.cpp:114-155): frame 0 to the origin and the identity rotation; mutates
  // the map's frame poses and point locations.
  void Normalize(sg_map* m);

 private:
  void Upload(const sg_map* m);
  void Download(sg_map* m, bool X, bool unc);
  sg_device_options dev_;
  hipStream_t stream_ = nullptr;
  bool own_stream_ = false;
  HostIo io_;   // uploads / downloads without a copy engine (hostio.h)
  int P_ = 0, M_ = 0;
  int32_t counters_h_[2] = {1, 0};
  DBuf<double> k_, q_, t_, X_, unc_, obs_pt_, obs_err_;
  DBuf<int32_t> fcam_, flags_, obs_frame_, obs_dis_, poff_, pobs_, counters_;
  DBuf<uint8_t> cand_, changed_;
  DBuf<unsigned long long> scal_;
};

}  // namespace sg

#endif  // SG_MAP_OPS_H_
