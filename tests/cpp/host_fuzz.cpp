// tests/cpp/host_fuzz.cpp — host-only robustness driver for the engine's untrusted-input parsers and host logic,
// built with AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_host_sanitizers.py (the
// reference's only sanitizer hooks are its CMake flags, CMakeLists.txt:59-62).
//
//   * pba_map_load (pba_map.cpp): the reference's map.cereal (save_map_file, map_utils.h:58-86) and opt_calib.json
//     (serialization.h:115-143) — the valid fixture, every truncation point on a grid, and random byte mutations
//     (single bytes, 64-bit size tags overwritten with huge / boundary values, JSON characters replaced);
//   * pba_outlier_landmarks (pba_outliers_host.cpp): random observation lists, out-of-range ids included.
// Every call must return PBA_OK or a negative status without a sanitizer report; on PBA_OK every getter is called
// with arrays sized from pba_map_get_info.
//   usage: host_fuzz <map.cereal> <opt_calib.json> <tmp dir> <seed> <mutations>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "pba.h"
#include "pba_host.h"

namespace pba {
namespace detail {
thread_local std::string g_last_error;  // defined in pba_engine.hip in the full library
}  // namespace detail
}  // namespace pba

static std::string slurp(const char* p) {
  std::ifstream f(p, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}
static void spit(const std::string& p, const std::string& s) {
  std::ofstream f(p, std::ios::binary | std::ios::trunc);
  f.write(s.data(), (std::streamsize)s.size());
}

static long n_ok = 0, n_err = 0;

static void load_and_read(const std::string& map, const std::string& calib) {
  pba_map* m = nullptr;
  const int rc = pba_map_load(map.c_str(), calib.c_str(), &m);
  if (rc != PBA_OK) {
    ++n_err;
    if (m) { fprintf(stderr, "failed load returned a map\n"); abort(); }
    return;
  }
  ++n_ok;
  pba_map_info in{};
  if (pba_map_get_info(m, &in) != PBA_OK) abort();
  if (in.n_frames < 0 || in.n_points < 0 || in.n_blocks < 0 || in.n_cams < 0 || in.n_outlier_obs < 0) abort();
  std::vector<double> intr(8 * (size_t)in.n_cams + 1), tic(7 * (size_t)in.n_cams + 1), poses(7 * (size_t)in.n_frames + 1);
  std::vector<int64_t> fid(in.n_frames + 1), tid(in.n_points + 1);
  std::vector<int32_t> fcam(in.n_frames + 1), host(in.n_points + 1), bp(in.n_blocks + 1), bt(in.n_blocks + 1);
  std::vector<double> uref(2 * (size_t)in.n_points + 1), rho(in.n_points + 1), uobs(2 * (size_t)in.n_blocks + 1);
  std::vector<int32_t> op(in.n_outlier_obs + 1), of(in.n_outlier_obs + 1);
  std::vector<double> ouv(2 * (size_t)in.n_outlier_obs + 1);
  pba_map_get_cameras(m, intr.data(), tic.data());
  pba_map_get_frames(m, fid.data(), fcam.data(), poses.data());
  pba_map_get_points(m, tid.data(), host.data(), uref.data(), rho.data());
  pba_map_get_blocks(m, bp.data(), bt.data(), uobs.data());
  pba_map_get_outlier_obs(m, op.data(), of.data(), ouv.data());
  // the problem must be consistent enough for pba_set_*: indices in range
  for (int i = 0; i < in.n_points; ++i)
    if (host[i] < 0 || host[i] >= in.n_frames) { fprintf(stderr, "host out of range\n"); abort(); }
  for (int b = 0; b < in.n_blocks; ++b)
    if (bp[b] < 0 || bp[b] >= in.n_points || bt[b] < 0 || bt[b] >= in.n_frames) { fprintf(stderr, "block out of range\n"); abort(); }
  for (int i = 0; i < in.n_frames; ++i)
    if (fcam[i] < 0 || fcam[i] >= in.n_cams) { fprintf(stderr, "frame camera out of range\n"); abort(); }
  pba_map_destroy(m);
}

int main(int argc, char** argv) {
  if (argc != 6) return 1;
  const std::string map = slurp(argv[1]), calib = slurp(argv[2]), dir = argv[3];
  const unsigned seed = (unsigned)atoi(argv[4]);
  const int mutations = atoi(argv[5]);
  const std::string mp = dir + "/map.cereal", cp = dir + "/opt_calib.json";
  std::mt19937 rng(seed);
  // 1. the valid fixture
  spit(mp, map);
  spit(cp, calib);
  load_and_read(mp, cp);
  if (n_ok != 1) { fprintf(stderr, "valid fixture did not load: %s\n", pba::detail::g_last_error.c_str()); return 2; }
  // 2. truncations (map, then calibration)
  const size_t step_m = map.size() / 400 + 1, step_c = calib.size() / 200 + 1;
  for (size_t cut = 0; cut < map.size(); cut += step_m) {
    spit(mp, map.substr(0, cut));
    load_and_read(mp, cp);
  }
  spit(mp, map);
  for (size_t cut = 0; cut < calib.size(); cut += step_c) {
    spit(cp, calib.substr(0, cut));
    load_and_read(mp, cp);
  }
  spit(cp, calib);
  // 3. mutations
  const uint64_t sizes[] = {0ull, 1ull, 0x7fffffffull, 0xffffffffull, 0x100000000ull, ~0ull, 1ull << 62};
  const char jchars[] = "{}[]\":,0-.eE9 \\n";
  for (int it = 0; it < mutations; ++it) {
    std::string m2 = map, c2 = calib;
    const int kind = (int)(rng() % 4);
    if (kind == 0) {  // random bytes of the map
      const int n = 1 + (int)(rng() % 8);
      for (int j = 0; j < n; ++j) m2[rng() % m2.size()] = (char)(rng() & 255);
    } else if (kind == 1) {  // an 8-byte field overwritten with a size-tag extreme
      const size_t at = (rng() % (m2.size() / 8)) * 8;
      const uint64_t v = sizes[rng() % (sizeof(sizes) / sizeof(sizes[0]))];
      if (at + 8 <= m2.size()) memcpy(&m2[at], &v, 8);
    } else if (kind == 2) {  // JSON structure characters
      const int n = 1 + (int)(rng() % 4);
      for (int j = 0; j < n; ++j) c2[rng() % c2.size()] = jchars[rng() % (sizeof(jchars) - 1)];
    } else {  // a deleted span of the map
      const size_t a = rng() % m2.size(), len = 1 + rng() % 64;
      m2.erase(a, len);
    }
    spit(mp, m2);
    spit(cp, c2);
    load_and_read(mp, cp);
  }
  // 4. remove_outlier_landmarks on random inputs
  long outl_ok = 0, outl_err = 0;
  for (int it = 0; it < 2000; ++it) {
    const int np = (int)(rng() % 50), no = (int)(rng() % 200);
    std::vector<int32_t> pt(no), fr(no), cnt(5);
    std::vector<uint32_t> fl(no);
    std::vector<uint8_t> oo(no), rm(np + 1);
    for (int i = 0; i < no; ++i) {
      pt[i] = (int32_t)(rng() % (np + 2)) - (rng() % 16 == 0 ? 1 : 0);  // occasionally out of range
      fr[i] = (int32_t)(rng() % 30);
      fl[i] = rng() & 15;
      oo[i] = rng() % 5 == 0;
    }
    const int rc = pba_outlier_landmarks(np, no, pt.data(), fr.data(), fl.data(), rng() % 2 ? oo.data() : nullptr,
                                         rm.data(), rng() % 2 ? cnt.data() : nullptr);
    (rc == PBA_OK ? outl_ok : outl_err)++;
  }
  printf("{\"map_loads_ok\": %ld, \"map_loads_rejected\": %ld, \"outlier_ok\": %ld, \"outlier_rejected\": %ld}\n", n_ok,
         n_err, outl_ok, outl_err);
  return 0;
}
