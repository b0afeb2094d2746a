// pba_outliers_host.cpp — the host-only half of the outlier pass: remove_outlier_landmarks'
// per-track decision (src/sfm.cpp:2028-2114) on the flags pba_compute_projections (pba_outliers.hip) produced.
// Plain C++ (no HIP), so it also builds with the host sanitizers (tests/test_host_sanitizers.py).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

#include "pba.h"
#include "pba_host.h"

using pba::detail::fail;

extern "C" {

// remove_outlier_landmarks (sfm.cpp:2028-2114) on the flags of pba_compute_projections: host logic, no device.
int pba_outlier_landmarks(int32_t n_points, int32_t n_obs, const int32_t* obs_point, const int32_t* obs_frame,
                          const uint32_t* flags, const uint8_t* obs_is_outlier, uint8_t* remove, int32_t* counts) {
  if (n_points < 0 || n_obs < 0 || (n_obs > 0 && (!obs_point || !obs_frame || !flags)) || (n_points > 0 && !remove))
    return fail(PBA_ERR_INVALID_ARGUMENT, "bad outlier arguments");
  for (int i = 0; i < n_obs; ++i)
    if (obs_point[i] < 0 || obs_point[i] >= n_points) return fail(PBA_ERR_INVALID_ARGUMENT, "observation point out of range");
  // any observation with a flag other than the normal reprojection error (sfm.cpp:2040-2053)
  bool any_severe = false;
  for (int i = 0; i < n_obs && !any_severe; ++i)
    if (!(obs_is_outlier && obs_is_outlier[i]) && (flags[i] & ~(uint32_t)PBA_OUTLIER_REPROJECTION_NORMAL)) any_severe = true;
  // each track's inlier observations in FrameCamId (= frame index) order, as track_projections iterates
  std::vector<int> order(n_obs);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
    return obs_point[x] != obs_point[y] ? obs_point[x] < obs_point[y] : obs_frame[x] < obs_frame[y];
  });
  int n_huge = 0, n_normal = 0, n_dist = 0, n_z = 0;
  std::memset(remove, 0, (size_t)n_points);
  for (size_t s = 0; s < order.size();) {
    const int pt = obs_point[order[s]];
    size_t e = s;
    while (e < order.size() && obs_point[order[e]] == pt) ++e;
    bool rm = false, normal_counted = false;
    for (size_t q = s; q < e; ++q) {  // sfm.cpp:2058-2095, first decisive flag wins
      const int i = order[q];
      if (obs_is_outlier && obs_is_outlier[i]) continue;
      const uint32_t f = flags[i];
      if (f & PBA_OUTLIER_REPROJECTION_HUGE) { ++n_huge; rm = true; break; }
      if (f & PBA_OUTLIER_REPROJECTION_NORMAL) {
        if (!normal_counted) { ++n_normal; normal_counted = true; }
        if (!any_severe) { rm = true; break; }
      }
      if (f & PBA_OUTLIER_CAMERA_DISTANCE) { rm = true; ++n_dist; break; }
      if (f & PBA_OUTLIER_Z_COORDINATE) { rm = true; ++n_z; break; }
    }
    remove[pt] = rm ? 1 : 0;
    s = e;
  }
  if (counts) {
    counts[0] = n_huge;
    counts[1] = n_normal;
    counts[2] = n_dist;
    counts[3] = n_z;
    counts[4] = any_severe ? 1 : 0;
  }
  return PBA_OK;
}

}  // extern "C"
