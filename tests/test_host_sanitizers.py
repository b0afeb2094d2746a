"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (the reference's own sanitizer hooks
are only its CMake flags, CMakeLists.txt:59-62).  pba_map.cpp parses untrusted files in the format of
map_utils.h:89-116 / serialization.h:115-205, and pba_outliers_host.cpp is the host logic of
remove_outlier_landmarks (sfm.cpp:2028-2114).  Both are plain C++ (pba_host.h, no HIP), so g++ builds them with
-fsanitize=address,undefined -fno-sanitize-recover=all together with tests/cpp/host_fuzz.cpp, which feeds the map
fixture of tests/golden/map_small/ whole, truncated at ~600 points and mutated 3000 times.  Any sanitizer report
aborts the driver (non-zero exit)."""
import json
import os
import subprocess
import tempfile

from helpers import ROOT

CSRC = os.path.join(ROOT, "photometric-bundle-adjustment_amd", "csrc")
MAP = os.path.join(ROOT, "tests", "golden", "map_small")


def test_map_loader_and_outlier_logic_under_asan_ubsan():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "host_fuzz")
        cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
               "-fno-sanitize-recover=all", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
               os.path.join(CSRC, "pba_map.cpp"), os.path.join(CSRC, "pba_outliers_host.cpp"),
               os.path.join(ROOT, "tests", "cpp", "host_fuzz.cpp"), "-o", exe]
        subprocess.run(cmd, check=True, capture_output=True, text=True)
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
        env.pop("LD_PRELOAD", None)
        r = subprocess.run([exe, os.path.join(MAP, "map.cereal"), os.path.join(MAP, "opt_calib.json"), td, "7", "3000"],
                           capture_output=True, text=True, env=env, timeout=600)
        assert r.returncode == 0, r.stderr[-6000:]
        out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["map_loads_ok"] >= 1 and out["map_loads_rejected"] >= 100, out
    assert out["outlier_ok"] > 0 and out["outlier_rejected"] > 0, out
