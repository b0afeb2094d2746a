// pba_map.cpp — problem loader from the reference's on-disk formats, host-only C++.
//
//   map.cereal      cereal BinaryOutputArchive written by save_map_file (include/visnav/map_utils.h:58-86):
//                   feature_corners, feature_matches, feature_tracks, outlier_tracks, cameras, landmarks, with the
//                   serializers of include/visnav/serialization.h:155-205 and cereal's std containers
//                   (map-likes: uint64 size + key/value items; vectors of arithmetic: uint64 size + raw bytes;
//                   other vectors: uint64 size + items; std::bitset in binary archives: uint8 type (3 = bits)
//                   + ⌈N/8⌉ bytes; little-endian, no padding).
//   opt_calib.json  cereal JSONOutputArchive of Calibration (serialization.h:115-143, 161-164): "cam.T_i_c" poses
//                   {px py pz qx qy qz qw} and "cam.intrinsics" {cam_type fx fy cx cy p1..p4 width height}; the
//                   LoadCalibration<DoubleSphereCamera> form {fx fy cx cy xi alpha} (serialization.h:102-113,
//                   data/euroc_calib/calibration-double-sphere.json) is accepted too.
//
// The problem is then built exactly like bundle_adjustment() (map_utils.h:322-375): one frame per map camera
// (FrameCamId order, pose T_w_c), one point per landmark (TrackId order) anchored at obs.begin() — the smallest
// FrameCamId (common_types.h:208) — with u_ref = that observation's corner and ρ = inv_depth, and one block per
// further observation (FrameCamId order) with u_obs = its corner.  Outlier observations are kept separately
// (for pba_compute_projections).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "pba.h"
#include "pba_host.h"

using pba::detail::fail;

namespace {

// ---- cereal binary reader -------------------------------------------------------------------------------
struct BinReader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  template <class T>
  T get() {
    T v{};
    if ((size_t)(end - p) < sizeof(T)) { ok = false; p = end; return v; }
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  void skip(uint64_t n) {
    if ((uint64_t)(end - p) < n) { ok = false; p = end; return; }
    p += n;
  }
  uint64_t size() {  // cereal size_tag (CEREAL_SIZE_TYPE = uint64_t), sanity-capped by the bytes left
    const uint64_t n = get<uint64_t>();
    if (n > (uint64_t)(end - p)) ok = false;
    return ok ? n : 0;
  }
};

struct FrameCamId {  // common_types.h:66-105 (frame_id int64, cam_id size_t), ordered by (frame, cam)
  int64_t frame;
  uint64_t cam;
  bool operator<(const FrameCamId& o) const { return frame != o.frame ? frame < o.frame : cam < o.cam; }
  bool operator==(const FrameCamId& o) const { return frame == o.frame && cam == o.cam; }
};
FrameCamId get_fcid(BinReader& r) {
  FrameCamId f;
  f.frame = r.get<int64_t>();
  f.cam = r.get<uint64_t>();
  return f;
}
void get_se3(BinReader& r, double* T) {  // serialize(SE3d): px py pz qx qy qz qw → storage [qx qy qz qw tx ty tz]
  double v[7];
  for (double& x : v) x = r.get<double>();
  T[0] = v[3]; T[1] = v[4]; T[2] = v[5]; T[3] = v[6];
  T[4] = v[0]; T[5] = v[1]; T[6] = v[2];
}
using Track = std::map<FrameCamId, int32_t>;  // FeatureTrack (common_types.h:175)
Track get_track(BinReader& r) {
  Track t;
  const uint64_t n = r.size();
  for (uint64_t i = 0; i < n && r.ok; ++i) {
    const FrameCamId f = get_fcid(r);
    t[f] = r.get<int32_t>();
  }
  return t;
}

struct Landmark {
  double inv_depth;
  Track obs, outlier_obs;
};

// ---- minimal JSON (cereal's JSON archive output) ----------------------------------------------------------
struct Json {
  enum Kind { NUL, NUM, STR, BOOL, ARR, OBJ } kind = NUL;
  double num = 0;
  std::string str;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;
  const Json* find(const std::string& k) const {
    for (const auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

struct JsonParser {
  const char* p;
  const char* end;
  bool ok = true;
  void ws() { while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
  bool lit(const char* s) {
    const size_t n = std::strlen(s);
    if ((size_t)(end - p) >= n && std::strncmp(p, s, n) == 0) { p += n; return true; }
    return false;
  }
  std::string string() {
    std::string s;
    if (p >= end || *p != '"') { ok = false; return s; }
    ++p;
    while (p < end && *p != '"') {
      if (*p == '\\' && p + 1 < end) { ++p; s.push_back(*p == 'n' ? '\n' : *p == 't' ? '\t' : *p); ++p; }
      else s.push_back(*p++);
    }
    if (p >= end) ok = false;
    else ++p;
    return s;
  }
  Json value(int depth = 0) {
    Json v;
    if (depth > 64) { ok = false; return v; }
    ws();
    if (p >= end) { ok = false; return v; }
    if (*p == '{') {
      ++p;
      v.kind = Json::OBJ;
      ws();
      if (p < end && *p == '}') { ++p; return v; }
      while (ok) {
        ws();
        std::string k = string();
        ws();
        if (p >= end || *p != ':') { ok = false; break; }
        ++p;
        v.obj.emplace_back(std::move(k), value(depth + 1));
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == '}') { ++p; break; }
        ok = false;
      }
    } else if (*p == '[') {
      ++p;
      v.kind = Json::ARR;
      ws();
      if (p < end && *p == ']') { ++p; return v; }
      while (ok) {
        v.arr.push_back(value(depth + 1));
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == ']') { ++p; break; }
        ok = false;
      }
    } else if (*p == '"') {
      v.kind = Json::STR;
      v.str = string();
    } else if (lit("true")) {
      v.kind = Json::BOOL; v.num = 1;
    } else if (lit("false")) {
      v.kind = Json::BOOL; v.num = 0;
    } else if (lit("null")) {
      v.kind = Json::NUL;
    } else {
      char* q = nullptr;
      const std::string tok(p, std::min<size_t>(64, (size_t)(end - p)));
      v.num = std::strtod(tok.c_str(), &q);
      if (q == tok.c_str()) { ok = false; return v; }
      p += q - tok.c_str();
      v.kind = Json::NUM;
    }
    return v;
  }
};

bool read_file(const char* path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

int model_of(const std::string& name) {  // camera_models.h getName(): "pinhole", "ds", "eucm", "kb4"
  if (name == "pinhole") return PBA_CAMERA_PINHOLE;
  if (name == "ds") return PBA_CAMERA_DOUBLE_SPHERE;
  if (name == "eucm") return PBA_CAMERA_EUCM;
  if (name == "kb4") return PBA_CAMERA_KB4;
  return -1;
}

}  // namespace

struct pba_map {
  pba_map_info info{};
  std::vector<double> intrinsics, T_i_c;
  std::vector<int64_t> frame_id;
  std::vector<int32_t> frame_cam;
  std::vector<double> poses;
  std::vector<int64_t> track_id;
  std::vector<int32_t> point_host;
  std::vector<double> u_ref, inv_dist;
  std::vector<int32_t> block_point, block_target;
  std::vector<double> u_obs;
  std::vector<int32_t> out_point, out_frame;
  std::vector<double> out_uv;
};

template <class T>
static void copy_out(const std::vector<T>& v, T* dst) {
  if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(T));
}

static int load_calib(const char* path, pba_map& m) {
  std::string txt;
  if (!read_file(path, txt)) return fail(PBA_ERR_INVALID_ARGUMENT, std::string("cannot read calibration ") + path);
  JsonParser jp{txt.data(), txt.data() + txt.size()};
  const Json root = jp.value();
  if (!jp.ok || root.kind != Json::OBJ) return fail(PBA_ERR_INVALID_ARGUMENT, "calibration: malformed JSON");
  const Json* v0 = root.find("value0");
  const Json* tic = v0 ? v0->find("cam.T_i_c") : nullptr;
  const Json* intr = v0 ? v0->find("cam.intrinsics") : nullptr;
  if (!intr || intr->kind != Json::ARR || intr->arr.empty())
    return fail(PBA_ERR_INVALID_ARGUMENT, "calibration: value0/cam.intrinsics missing");
  const int nc = (int)intr->arr.size();
  m.intrinsics.assign(8 * (size_t)nc, 0.0);
  m.T_i_c.assign(7 * (size_t)nc, 0.0);
  int model = -2;
  auto num = [](const Json& o, const char* k, double& out) {
    const Json* x = o.find(k);
    if (!x || x->kind != Json::NUM) return false;
    out = x->num;
    return true;
  };
  for (int c = 0; c < nc; ++c) {
    const Json& o = intr->arr[c];
    double* k = m.intrinsics.data() + 8 * c;
    int mc;
    const Json* ty = o.find("cam_type");
    if (ty && ty->kind == Json::STR) {  // save(shared_ptr<AbstractCamera>) form
      mc = model_of(ty->str);
      if (mc < 0) return fail(PBA_ERR_INVALID_ARGUMENT, "calibration: unsupported camera model " + ty->str);
      static const char* names[8] = {"fx", "fy", "cx", "cy", "p1", "p2", "p3", "p4"};
      for (int j = 0; j < 8; ++j)
        if (!num(o, names[j], k[j])) return fail(PBA_ERR_INVALID_ARGUMENT, std::string("calibration: missing ") + names[j]);
      double w = 0, h = 0;
      if (num(o, "width", w) && num(o, "height", h)) { m.info.width = (int32_t)w; m.info.height = (int32_t)h; }
    } else {  // LoadCalibration<DoubleSphereCamera> form (fx fy cx cy xi alpha)
      mc = PBA_CAMERA_DOUBLE_SPHERE;
      static const char* names[6] = {"fx", "fy", "cx", "cy", "xi", "alpha"};
      for (int j = 0; j < 6; ++j)
        if (!num(o, names[j], k[j])) return fail(PBA_ERR_INVALID_ARGUMENT, std::string("calibration: missing ") + names[j]);
    }
    if (model == -2) model = mc;
    else if (model != mc) return fail(PBA_ERR_INVALID_ARGUMENT, "calibration: cameras of different models");
    double* T = m.T_i_c.data() + 7 * c;
    T[3] = 1.0;
    if (tic && tic->kind == Json::ARR && c < (int)tic->arr.size()) {
      const Json& t = tic->arr[c];
      double v[7] = {0, 0, 0, 0, 0, 0, 1};
      static const char* names[7] = {"px", "py", "pz", "qx", "qy", "qz", "qw"};
      for (int j = 0; j < 7; ++j) num(t, names[j], v[j]);
      T[0] = v[3]; T[1] = v[4]; T[2] = v[5]; T[3] = v[6]; T[4] = v[0]; T[5] = v[1]; T[6] = v[2];
    }
  }
  m.info.n_cams = nc;
  m.info.camera_model = model;
  return PBA_OK;
}

static int load_map(const char* path, pba_map& m) {
  std::string buf;
  if (!read_file(path, buf)) return fail(PBA_ERR_INVALID_ARGUMENT, std::string("cannot read map ") + path);
  BinReader r{reinterpret_cast<const uint8_t*>(buf.data()), reinterpret_cast<const uint8_t*>(buf.data()) + buf.size()};
  // feature_corners: {FrameCamId → KeypointsData{corners, corner_angles, corner_descriptors}}
  std::map<FrameCamId, std::vector<double>> corners;
  const uint64_t n_img = r.size();
  for (uint64_t i = 0; i < n_img && r.ok; ++i) {
    const FrameCamId f = get_fcid(r);
    const uint64_t nc = r.size();  // vector<Vector2d>: items of 2 doubles (static Eigen size, no dims)
    std::vector<double>& c = corners[f];
    c.resize(2 * nc);
    for (uint64_t j = 0; j < 2 * nc && r.ok; ++j) c[j] = r.get<double>();
    r.skip(8 * r.size());  // corner_angles: vector<double>, raw
    const uint64_t nd = r.size();  // corner_descriptors: vector<bitset<256>>, each type byte + 32 bytes
    for (uint64_t j = 0; j < nd && r.ok; ++j) {
      const uint8_t type = r.get<uint8_t>();
      if (type != 3) return fail(PBA_ERR_INVALID_ARGUMENT, "map: unexpected bitset encoding");
      r.skip(32);
    }
  }
  // feature_matches: {(FrameCamId, FrameCamId) → MatchData{T_i_j, inliers, matches}} — skipped
  const uint64_t n_match = r.size();
  for (uint64_t i = 0; i < n_match && r.ok; ++i) {
    r.skip(32 + 56);
    r.skip(8 * r.size());  // inliers: vector<pair<int,int>>
    r.skip(8 * r.size());  // matches
  }
  // feature_tracks, outlier_tracks: {TrackId → FeatureTrack} — skipped
  for (int t = 0; t < 2 && r.ok; ++t) {
    const uint64_t n = r.size();
    for (uint64_t i = 0; i < n && r.ok; ++i) {
      r.skip(8);
      r.skip(20 * r.size());
    }
  }
  // cameras: {FrameCamId → Camera{T_w_c}}
  std::map<FrameCamId, int> frame_index;
  const uint64_t n_cam = r.size();
  for (uint64_t i = 0; i < n_cam && r.ok; ++i) {
    const FrameCamId f = get_fcid(r);
    double T[7];
    get_se3(r, T);
    frame_index[f] = 0;
    m.poses.insert(m.poses.end(), T, T + 7);
    m.frame_id.push_back(f.frame);
    m.frame_cam.push_back((int32_t)f.cam);
  }
  // landmarks: {TrackId → Landmark{inv_depth, obs, outlier_obs}}
  std::map<int64_t, Landmark> lms;
  const uint64_t n_lm = r.size();
  for (uint64_t i = 0; i < n_lm && r.ok; ++i) {
    const int64_t id = r.get<int64_t>();
    Landmark l;
    l.inv_depth = r.get<double>();
    l.obs = get_track(r);
    l.outlier_obs = get_track(r);
    lms[id] = std::move(l);
  }
  if (!r.ok) return fail(PBA_ERR_INVALID_ARGUMENT, "map: truncated or malformed cereal archive");
  // frames in FrameCamId order (the Cameras std::map order); poses were read in that order already
  {
    std::vector<std::pair<FrameCamId, int>> fr;
    for (size_t i = 0; i < m.frame_id.size(); ++i) fr.push_back({FrameCamId{m.frame_id[i], (uint64_t)m.frame_cam[i]}, (int)i});
    int idx = 0;
    for (auto& kv : frame_index) kv.second = idx++;
    std::vector<double> poses(m.poses.size());
    for (auto& f : fr) std::memcpy(&poses[7 * frame_index[f.first]], &m.poses[7 * f.second], 7 * sizeof(double));
    m.poses.swap(poses);
    m.frame_id.clear();
    m.frame_cam.clear();
    for (auto& kv : frame_index) {
      m.frame_id.push_back(kv.first.frame);
      m.frame_cam.push_back((int32_t)kv.first.cam);
    }
  }
  auto corner = [&](const FrameCamId& f, int fid, double* uv) -> bool {
    auto it = corners.find(f);
    if (it == corners.end() || fid < 0 || 2 * (size_t)fid + 1 >= it->second.size()) return false;
    uv[0] = it->second[2 * fid];
    uv[1] = it->second[2 * fid + 1];
    return true;
  };
  for (const auto& kv : lms) {
    const Landmark& l = kv.second;
    if (l.obs.empty()) continue;
    const int pt = (int)m.track_id.size();
    const FrameCamId& h = l.obs.begin()->first;  // anchor = smallest FrameCamId (common_types.h:208)
    auto hit = frame_index.find(h);
    if (hit == frame_index.end()) return fail(PBA_ERR_INVALID_ARGUMENT, "map: landmark observed by a frame not in the map");
    double uv[2];
    if (!corner(h, l.obs.begin()->second, uv)) return fail(PBA_ERR_INVALID_ARGUMENT, "map: observation without corner");
    m.track_id.push_back(kv.first);
    m.point_host.push_back(hit->second);
    m.u_ref.insert(m.u_ref.end(), uv, uv + 2);
    m.inv_dist.push_back(l.inv_depth);
    for (auto it = std::next(l.obs.begin()); it != l.obs.end(); ++it) {  // map_utils.h:355-373
      auto fi = frame_index.find(it->first);
      if (fi == frame_index.end()) return fail(PBA_ERR_INVALID_ARGUMENT, "map: landmark observed by a frame not in the map");
      if (!corner(it->first, it->second, uv)) return fail(PBA_ERR_INVALID_ARGUMENT, "map: observation without corner");
      m.block_point.push_back(pt);
      m.block_target.push_back(fi->second);
      m.u_obs.insert(m.u_obs.end(), uv, uv + 2);
    }
    for (const auto& o : l.outlier_obs) {
      auto fi = frame_index.find(o.first);
      if (fi == frame_index.end() || !corner(o.first, o.second, uv)) continue;
      m.out_point.push_back(pt);
      m.out_frame.push_back(fi->second);
      m.out_uv.insert(m.out_uv.end(), uv, uv + 2);
    }
  }
  m.info.n_frames = (int32_t)m.frame_cam.size();
  m.info.n_points = (int32_t)m.track_id.size();
  m.info.n_blocks = (int32_t)m.block_point.size();
  m.info.n_outlier_obs = (int32_t)m.out_point.size();
  return PBA_OK;
}

extern "C" {

int pba_map_load(const char* map_path, const char* calib_path, pba_map** out) {
  if (!map_path || !calib_path || !out) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  std::unique_ptr<pba_map> m(new pba_map());
  if (int rc = load_calib(calib_path, *m)) return rc;
  if (int rc = load_map(map_path, *m)) return rc;
  for (int32_t c : m->frame_cam)
    if (c < 0 || c >= m->info.n_cams) return fail(PBA_ERR_INVALID_ARGUMENT, "map: camera id beyond the calibration");
  *out = m.release();
  return PBA_OK;
}

int pba_map_destroy(pba_map* m) {
  delete m;
  return PBA_OK;
}

int pba_map_get_info(const pba_map* m, pba_map_info* info) {
  if (!m || !info) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  *info = m->info;
  return PBA_OK;
}

int pba_map_get_cameras(const pba_map* m, double* intrinsics, double* T_i_c) {
  if (!m) return fail(PBA_ERR_INVALID_ARGUMENT, "null map");
  copy_out(m->intrinsics, intrinsics);
  copy_out(m->T_i_c, T_i_c);
  return PBA_OK;
}

int pba_map_get_frames(const pba_map* m, int64_t* frame_id, int32_t* frame_cam, double* poses) {
  if (!m) return fail(PBA_ERR_INVALID_ARGUMENT, "null map");
  copy_out(m->frame_id, frame_id);
  copy_out(m->frame_cam, frame_cam);
  copy_out(m->poses, poses);
  return PBA_OK;
}

int pba_map_get_points(const pba_map* m, int64_t* track_id, int32_t* host_frame, double* u_ref, double* inv_dist) {
  if (!m) return fail(PBA_ERR_INVALID_ARGUMENT, "null map");
  copy_out(m->track_id, track_id);
  copy_out(m->point_host, host_frame);
  copy_out(m->u_ref, u_ref);
  copy_out(m->inv_dist, inv_dist);
  return PBA_OK;
}

int pba_map_get_blocks(const pba_map* m, int32_t* block_point, int32_t* block_target, double* u_obs) {
  if (!m) return fail(PBA_ERR_INVALID_ARGUMENT, "null map");
  copy_out(m->block_point, block_point);
  copy_out(m->block_target, block_target);
  copy_out(m->u_obs, u_obs);
  return PBA_OK;
}

int pba_map_get_outlier_obs(const pba_map* m, int32_t* point, int32_t* frame, double* uv) {
  if (!m) return fail(PBA_ERR_INVALID_ARGUMENT, "null map");
  copy_out(m->out_point, point);
  copy_out(m->out_frame, frame);
  copy_out(m->out_uv, uv);
  return PBA_OK;
}

}  // extern "C"
