// oracle/map_writer.cpp — TEST INFRASTRUCTURE ONLY (fixture generator, built into oracle/_ref/ by oracle/Makefile).
//
// Writes a small synthetic stereo map in the reference's on-disk formats with the reference's own vendored
// cereal library (thirdparty/cereal), so that the product's loader (csrc/pba_map.cpp) is pinned by cereal's
// actual encoding rather than by our reading of it:
//   map.cereal      save_map_file order (include/visnav/map_utils.h:58-86): corners, matches, tracks,
//                   outlier tracks, cameras, landmarks.  The types restate include/visnav/common_types.h with
//                   std::unordered_map in place of tbb::concurrent_unordered_map (TBB is absent here) — cereal
//                   serialises both through the same generic map-like path (size tag + key/value items).
//                   Serializers restate include/visnav/serialization.h:148-205 (field order and names).
//   opt_calib.json  Calibration as written by calibration.cpp:431-435 (serialization.h:115-143, 161-164).
//   expect.bin      the problem bundle_adjustment() would build (map_utils.h:322-375), in the loader's order.
#include <bitset>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <map>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include <Eigen/Dense>
#include <Eigen/StdVector>
#include <sophus/se3.hpp>

#include <cereal/archives/binary.hpp>
#include <cereal/archives/json.hpp>
#include <cereal/cereal.hpp>
#include <cereal/types/bitset.hpp>
#include <cereal/types/map.hpp>
#include <cereal/types/string.hpp>
#include <cereal/types/unordered_map.hpp>
#include <cereal/types/utility.hpp>
#include <cereal/types/vector.hpp>

namespace mw {
using FrameId = int64_t;
using CamId = std::size_t;
struct FrameCamId {
  FrameId frame_id = 0;
  CamId cam_id = 0;
  bool operator==(const FrameCamId& o) const { return frame_id == o.frame_id && cam_id == o.cam_id; }
  bool operator<(const FrameCamId& o) const { return frame_id == o.frame_id ? cam_id < o.cam_id : frame_id < o.frame_id; }
};
struct FcidHash {
  size_t operator()(const FrameCamId& f) const { return std::hash<int64_t>()(f.frame_id * 2 + (int64_t)f.cam_id); }
};
struct PairHash {
  size_t operator()(const std::pair<FrameCamId, FrameCamId>& p) const { return FcidHash()(p.first) * 31 + FcidHash()(p.second); }
};
using FeatureId = int;
using TrackId = int64_t;
struct KeypointsData {
  std::vector<Eigen::Vector2d, Eigen::aligned_allocator<Eigen::Vector2d>> corners;
  std::vector<double> corner_angles;
  std::vector<std::bitset<256>> corner_descriptors;
};
using Corners = std::unordered_map<FrameCamId, KeypointsData, FcidHash>;
struct MatchData {
  Sophus::SE3d T_i_j;
  std::vector<std::pair<FeatureId, FeatureId>> matches, inliers;
};
using Matches = std::unordered_map<std::pair<FrameCamId, FrameCamId>, MatchData, PairHash>;
using FeatureTrack = std::map<FrameCamId, FeatureId>;
using FeatureTracks = std::unordered_map<TrackId, FeatureTrack>;
struct Camera {
  Sophus::SE3d T_w_c;
};
using Cameras = std::map<FrameCamId, Camera>;
struct Landmark {
  double inv_depth = 1;
  FeatureTrack obs, outlier_obs;
};
using Landmarks = std::unordered_map<TrackId, Landmark>;
struct CamRec {  // what save(shared_ptr<AbstractCamera<double>>) writes (serialization.h:115-125)
  std::string cam_type;
  double intr[8];
  int width, height;
};
struct Calibration {
  std::vector<Sophus::SE3d, Eigen::aligned_allocator<Sophus::SE3d>> T_i_c;
  std::vector<CamRec> intrinsics;
};
}  // namespace mw

namespace cereal {
template <class Archive>
void serialize(Archive& ar, Eigen::Vector2d& m) {  // serialization.h:57-68 (static size: no dims)
  ar(m[0], m[1]);
}
template <class Archive>
void serialize(Archive& ar, Sophus::SE3d& p) {  // serialization.h:152-160
  ar(cereal::make_nvp("px", p.translation()[0]), cereal::make_nvp("py", p.translation()[1]),
     cereal::make_nvp("pz", p.translation()[2]), cereal::make_nvp("qx", p.so3().data()[0]),
     cereal::make_nvp("qy", p.so3().data()[1]), cereal::make_nvp("qz", p.so3().data()[2]),
     cereal::make_nvp("qw", p.so3().data()[3]));
}
template <class Archive>
void save(Archive& ar, const mw::CamRec& c) {  // serialization.h:115-125
  ar(cereal::make_nvp("cam_type", c.cam_type), cereal::make_nvp("fx", c.intr[0]), cereal::make_nvp("fy", c.intr[1]),
     cereal::make_nvp("cx", c.intr[2]), cereal::make_nvp("cy", c.intr[3]), cereal::make_nvp("p1", c.intr[4]),
     cereal::make_nvp("p2", c.intr[5]), cereal::make_nvp("p3", c.intr[6]), cereal::make_nvp("p4", c.intr[7]),
     cereal::make_nvp("width", c.width), cereal::make_nvp("height", c.height));
}
template <class Archive>
void serialize(Archive& ar, mw::Calibration& cam) {  // serialization.h:161-164 (CEREAL_NVP(cam.…) names)
  ar(cereal::make_nvp("cam.T_i_c", cam.T_i_c), cereal::make_nvp("cam.intrinsics", cam.intrinsics));
}
template <class Archive>
void serialize(Archive& ar, mw::MatchData& m) {  // serialization.h:172-175
  ar(CEREAL_NVP(m.T_i_j), CEREAL_NVP(m.inliers), CEREAL_NVP(m.matches));
}
template <class Archive>
void serialize(Archive& ar, mw::KeypointsData& m) {  // serialization.h:182-186
  ar(CEREAL_NVP(m.corners), CEREAL_NVP(m.corner_angles), CEREAL_NVP(m.corner_descriptors));
}
template <class Archive>
void serialize(Archive& ar, mw::Camera& c) {  // serialization.h:188-191
  ar(CEREAL_NVP(c.T_w_c));
}
template <class Archive>
void serialize(Archive& ar, mw::Landmark& lm) {  // serialization.h:193-196
  ar(CEREAL_NVP(lm.inv_depth), CEREAL_NVP(lm.obs), CEREAL_NVP(lm.outlier_obs));
}
template <class Archive>
void serialize(Archive& ar, mw::FrameCamId& f) {  // serialization.h:198-201
  ar(f.frame_id, f.cam_id);
}
}  // namespace cereal

using namespace mw;

// double sphere projection / unprojection (camera_models.h:226-277), for the synthetic scene only
static bool ds_project(const double* k, const Eigen::Vector3d& p, Eigen::Vector2d& uv) {
  const double xi = k[4], al = k[5];
  const double d1 = p.norm(), kk = xi * d1 + p.z(), d2 = std::sqrt(p.x() * p.x() + p.y() * p.y() + kk * kk);
  const double den = al * d2 + (1 - al) * kk;
  if (p.z() < 0.2 || den <= 0) return false;
  uv << k[0] * p.x() / den + k[2], k[1] * p.y() / den + k[3];
  return true;
}
static Eigen::Vector3d ds_unproject(const double* k, const Eigen::Vector2d& uv) {
  const double xi = k[4], al = k[5];
  const double mx = (uv.x() - k[2]) / k[0], my = (uv.y() - k[3]) / k[1], r2 = mx * mx + my * my;
  const double mz = (1 - al * al * r2) / (al * std::sqrt(1 - (2 * al - 1) * r2) + 1 - al);
  const double f = (mz * xi + std::sqrt(mz * mz + (1 - xi * xi) * r2)) / (mz * mz + r2);
  return Eigen::Vector3d(f * mx, f * my, f * mz - xi).normalized();
}

template <class T>
static void put(std::ofstream& o, const std::vector<T>& v) {
  const uint64_t n = v.size();
  o.write(reinterpret_cast<const char*>(&n), 8);
  o.write(reinterpret_cast<const char*>(v.data()), n * sizeof(T));
}

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: map_writer <out_dir> [frames] [landmarks] [seed]\n"); return 2; }
  const std::string dir = argv[1];
  const int F = argc > 2 ? std::atoi(argv[2]) : 12, NL = argc > 3 ? std::atoi(argv[3]) : 400;
  std::mt19937 rng(argc > 4 ? std::atoi(argv[4]) : 42);
  std::normal_distribution<double> N01(0, 1);
  std::uniform_real_distribution<double> U01(0, 1);
  const int W = 752, H = 480;
  Calibration calib;
  const double K[2][8] = {{370.34, 370.34, 375.5, 239.5, -0.05, 0.57, 0, 0}, {361.92, 361.92, 376.5, 240.5, -0.04, 0.56, 0, 0}};
  for (int c = 0; c < 2; ++c) {
    CamRec r{"ds", {}, W, H};
    for (int j = 0; j < 8; ++j) r.intr[j] = K[c][j];
    calib.intrinsics.push_back(r);
    calib.T_i_c.push_back(Sophus::SE3d(Sophus::SO3d::exp(Eigen::Vector3d(0, 0.01 * c, 0)), Eigen::Vector3d(0.11 * c, 0, 0)));
  }
  Cameras cameras;
  for (int f = 0; f < F; ++f) {
    const Sophus::SE3d T_w_i(Sophus::SO3d::exp(Eigen::Vector3d(0.01 * N01(rng), 0.03 * f, 0.01 * N01(rng))),
                             Eigen::Vector3d(0.15 * f, 0.02 * N01(rng), 0.02 * N01(rng)));
    for (int c = 0; c < 2; ++c) cameras[FrameCamId{f, (CamId)c}].T_w_c = T_w_i * calib.T_i_c[c];
  }
  Corners corners;
  for (auto& kv : cameras) corners[kv.first];  // every image has a corner list
  auto add_corner = [&](const FrameCamId& f, const Eigen::Vector2d& uv) {
    KeypointsData& kd = corners[f];
    kd.corners.push_back(uv);
    kd.corner_angles.push_back(U01(rng) * 6.28);
    std::bitset<256> b;
    for (int i = 0; i < 256; ++i) b[i] = U01(rng) < 0.5;
    kd.corner_descriptors.push_back(b);
    return (FeatureId)kd.corners.size() - 1;
  };
  Landmarks landmarks;
  FeatureTracks tracks, outlier_tracks;
  for (int l = 0; l < NL; ++l) {
    const Eigen::Vector3d pw(0.15 * F * U01(rng) - 0.5, 3.0 * (U01(rng) - 0.5), 4.0 + 4.0 * U01(rng));
    Landmark lm;
    for (auto& kv : cameras) {
      Eigen::Vector2d uv;
      if (!ds_project(K[kv.first.cam_id], kv.second.T_w_c.inverse() * pw, uv)) continue;
      if (uv.x() < 2 || uv.y() < 2 || uv.x() > W - 3 || uv.y() > H - 3 || U01(rng) < 0.4) continue;
      const bool corrupt = U01(rng) < 0.03, out = U01(rng) < 0.04;
      uv += Eigen::Vector2d(0.5 * N01(rng), 0.5 * N01(rng)) + (corrupt ? Eigen::Vector2d(25 * N01(rng), 25 * N01(rng)) : Eigen::Vector2d::Zero());
      const FeatureId fid = add_corner(kv.first, uv);
      (out && !lm.obs.empty() ? lm.outlier_obs : lm.obs)[kv.first] = fid;
      if (lm.obs.size() >= 6) break;
    }
    if (lm.obs.size() < 2) continue;
    const FrameCamId& h = lm.obs.begin()->first;
    const Eigen::Vector3d ph = cameras[h].T_w_c.inverse() * pw;
    lm.inv_depth = (1.0 / ph.norm()) * (1.0 + 0.02 * N01(rng));
    const TrackId id = 1000 + 7 * l;
    FeatureTrack t = lm.obs;
    t.insert(lm.outlier_obs.begin(), lm.outlier_obs.end());
    tracks[id] = t;
    landmarks[id] = lm;
    (void)ds_unproject;
  }
  for (int i = 0; i < 5; ++i) outlier_tracks[5 + i] = FeatureTrack{{FrameCamId{i, 0}, 0}};
  for (auto& kv : corners)  // clutter features that belong to no landmark
    for (int i = 0; i < 3; ++i) add_corner(kv.first, Eigen::Vector2d(U01(rng) * W, U01(rng) * H));
  Matches matches;
  for (int f = 0; f + 1 < F; ++f) {
    MatchData md;
    md.T_i_j = calib.T_i_c[0].inverse() * calib.T_i_c[1];
    for (int i = 0; i < 7; ++i) md.matches.push_back({i, i + 1});
    for (int i = 0; i < 4; ++i) md.inliers.push_back({i, i + 1});
    matches[{FrameCamId{f, 0}, FrameCamId{f, 1}}] = md;
  }
  {
    std::ofstream os(dir + "/map.cereal", std::ios::binary);
    cereal::BinaryOutputArchive archive(os);
    archive(corners);
    archive(matches);
    archive(tracks);
    archive(outlier_tracks);
    archive(cameras);
    archive(landmarks);
  }
  {
    std::ofstream os(dir + "/opt_calib.json");
    cereal::JSONOutputArchive archive(os);
    archive(calib);
  }
  // expected problem, in the loader's order (frames: FrameCamId order; points: TrackId order)
  std::map<FrameCamId, int> fidx;
  std::vector<int32_t> frame_cam;
  std::vector<double> poses;
  for (auto& kv : cameras) {
    fidx[kv.first] = (int)frame_cam.size();
    frame_cam.push_back((int32_t)kv.first.cam_id);
    const Sophus::SE3d& T = kv.second.T_w_c;
    const double v[7] = {T.so3().data()[0], T.so3().data()[1], T.so3().data()[2], T.so3().data()[3],
                         T.translation()[0], T.translation()[1], T.translation()[2]};
    poses.insert(poses.end(), v, v + 7);
  }
  std::map<TrackId, const Landmark*> sorted;
  for (auto& kv : landmarks) sorted[kv.first] = &kv.second;
  std::vector<int64_t> track_id;
  std::vector<int32_t> host, bp, bt, op, of;
  std::vector<double> u_ref, rho, u_obs, ouv;
  for (auto& kv : sorted) {
    const Landmark& lm = *kv.second;
    const int pt = (int)track_id.size();
    track_id.push_back(kv.first);
    auto it = lm.obs.begin();
    host.push_back(fidx[it->first]);
    const Eigen::Vector2d& ur = corners[it->first].corners[it->second];
    u_ref.push_back(ur.x());
    u_ref.push_back(ur.y());
    rho.push_back(lm.inv_depth);
    for (++it; it != lm.obs.end(); ++it) {
      const Eigen::Vector2d& uv = corners[it->first].corners[it->second];
      bp.push_back(pt);
      bt.push_back(fidx[it->first]);
      u_obs.push_back(uv.x());
      u_obs.push_back(uv.y());
    }
    for (auto& o : lm.outlier_obs) {
      const Eigen::Vector2d& uv = corners[o.first].corners[o.second];
      op.push_back(pt);
      of.push_back(fidx[o.first]);
      ouv.push_back(uv.x());
      ouv.push_back(uv.y());
    }
  }
  std::vector<double> intr;
  for (auto& c : calib.intrinsics) intr.insert(intr.end(), c.intr, c.intr + 8);
  std::ofstream ex(dir + "/expect.bin", std::ios::binary);
  put(ex, intr);
  put(ex, frame_cam);
  put(ex, poses);
  put(ex, track_id);
  put(ex, host);
  put(ex, u_ref);
  put(ex, rho);
  put(ex, bp);
  put(ex, bt);
  put(ex, u_obs);
  put(ex, op);
  put(ex, of);
  put(ex, ouv);
  std::printf("map: %zu frames, %zu landmarks, %zu blocks, %zu outlier obs\n", frame_cam.size(), track_id.size(),
              bp.size(), op.size());
  return 0;
}
