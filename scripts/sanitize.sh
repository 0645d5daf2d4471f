#!/bin/bash
# Host-side sanitizer run (SURVEY.md §5 "Race detection / sanitizers"): the C ABI's
# host code -- OBJ/MTL reader, CreateGeometry, KD build, KD cache, model
# descriptors (csrc/capi.cpp, host_model.cpp, kd_cache.cpp) -- built with
# AddressSanitizer + UndefinedBehaviorSanitizer (-fno-sanitize-recover: the
# first report fails the run) and driven by tests/cpp/sanitize_driver.cpp over
# the bundled scenes, the C4 mesh, a malformed OBJ/MTL corpus and forged KD-cache
# files.  CPU only: the HIP kernels are linked (unsanitized) but never launched.
#   scripts/sanitize.sh [build dir]    (default /tmp/mcpt_sanitize)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=${1:-/tmp/mcpt_sanitize}
mkdir -p "$B/corpus"
CSRC=$ROOT/montecarlopathtracer_amd/csrc
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -O1"
COMMON="-std=c++17 -fPIC -ffp-contract=off -I$ROOT/include"

# kernels: as shipped (device code is not sanitized; nothing launches them here)
for k in render wavefront; do
  [ "$B/$k.o" -nt "$CSRC/$k.hip" ] || $HIPCC -x hip --offload-arch=gfx950 -O3 $COMMON -c "$CSRC/$k.hip" -o "$B/$k.o"
done
# host code with ASan + UBSan
g++ $SAN $COMMON -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
    "$CSRC/capi.cpp" "$CSRC/host_model.cpp" "$CSRC/kd_cache.cpp" "$ROOT/tests/cpp/sanitize_driver.cpp" \
    "$B/render.o" "$B/wavefront.o" -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -o "$B/sanitize_driver"

# malformed OBJ/MTL corpus
python3 - "$B/corpus" <<'EOF'
import os, random, sys
d = sys.argv[1]
tri = "v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\n"
mtl = "newmtl m\nKd 0.5 0.5 0.5\nKa 1 1 1\n"
cases = {
    "empty.obj": "",
    "comments.obj": "# only\n#comments\n",
    "short_vertex.obj": "v 1 2\nv\nvn 0\nf 1 2 3\n",
    "two_vertex_face.obj": tri + "f 1//1 2//1\n",
    "zero_index.obj": tri + "f 0//1 1//1 2//1\n",
    "negative_index.obj": tri + "f -1//1 -2//1 -3//1\n",
    "index_past_end.obj": tri + "f 1//1 2//1 99//1\n",
    "huge_index.obj": tri + "f 1//1 2//1 99999999999999999999//1\n",
    "normal_past_end.obj": tri + "f 1//7 2//1 3//1\n",
    "missing_normal.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n",
    "bad_face_token.obj": tri + "f 1//1 x 3//1\n",
    "slashes.obj": tri + "f 1/ 2// //3\n",
    "numbers.obj": "v nan inf -inf\nv 1e999 -1e999 1e-999\nv 0x1p3 1 1\nvn 0 0 1\nf 1//1 2//1 3//1\n",
    "crlf_no_newline.obj": tri.replace("\n", "\r\n") + "f 1//1 2//1 3//1",
    "continuation.obj": "v 0 0 \\\n0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nf 1//1 2//1 \\\n3//1\n\\",
    "ngon.obj": "".join(f"v {i} {i % 7} {i % 3}\n" for i in range(1, 1001)) + "vn 0 0 1\nf " +
                " ".join(f"{i}//1" for i in range(1, 1001)) + "\n",
    "long_line.obj": tri + "g " + "x" * 200000 + "\nf 1//1 2//1 3//1\n",
    "keywords_only.obj": "g\nusemtl\nmtllib\nv\nvn\nvt\nf\n",
    "mtllib_missing.obj": "mtllib does_not_exist.mtl\n" + tri + "f 1//1 2//1 3//1\n",
    "mtllib_dir.obj": "mtllib .\n" + tri + "f 1//1 2//1 3//1\n",
    "bad.mtl": "newmtl\nKd\nKa 1\nNs x\nTr\nNi 1e999\nnewmtl b\nKs 1 1 1\n",
    "bad_mtl.obj": "mtllib bad.mtl\nusemtl b\n" + tri + "f 1//1 2//1 3//1\nusemtl nope\nf 3//1 2//1 1//1\n",
    "good.mtl": mtl,
    "degenerate.obj": "mtllib good.mtl\nusemtl m\n" + "v 0 0 0\n" * 3 + "vn 0 0 1\nf 1//1 2//1 3//1\n" * 70,
    "flat_many.obj": "mtllib good.mtl\nusemtl m\n" + "".join(
        f"v {i} 0 0\nv {i} 1 0\nv {i + 1} 0 0\n" for i in range(100)) + "vn 0 0 1\n" +
        "".join(f"f {3 * i + 1}//1 {3 * i + 2}//1 {3 * i + 3}//1\n" for i in range(100)),
}
r = random.Random(7)
cases["binary.obj"] = bytes(r.randrange(256) for _ in range(4096))
for name, text in cases.items():
    with open(os.path.join(d, name), "wb") as f:
        f.write(text if isinstance(text, bytes) else text.encode())
EOF
# mutated copies of a real scene: truncations and byte flips of scene01.obj
SCENE01=$(cd "$ROOT" && python3 -c "from montecarlopathtracer_amd.scenes import scene_path; print(scene_path('scene01'))")
python3 - "$B/corpus" "$SCENE01" <<'EOF'
import os, random, shutil, sys
d, src = sys.argv[1], sys.argv[2]
data = open(src, "rb").read()
shutil.copy(os.path.splitext(src)[0] + ".mtl", os.path.join(d, "scene01.mtl"))
r = random.Random(11)
for i in range(24):
    b = bytearray(data[: r.randrange(len(data))] if i % 2 else data)
    for _ in range(r.randrange(1, 40)):
        b[r.randrange(len(b))] = r.choice(b"0123456789/-+. \n\\fvgxe")
    open(os.path.join(d, f"scene01_mut{i:02d}.obj"), "wb").write(bytes(b))
EOF

SCENES=$(cd "$ROOT" && python3 -c "
from montecarlopathtracer_amd.scenes import scene_path
print(' '.join(scene_path(s) for s in ('scene01', 'scene02', 'scene03', 'cornell_bunny70k')))")
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=1:strict_string_checks=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export LSAN_OPTIONS=suppressions=$ROOT/scripts/lsan.supp
# the driver runs with a memory watchdog (ASan's shadow makes ulimit -v unusable):
# a KD build that ran away once took 45 GB before it was stopped
"$B/sanitize_driver" "$B" $SCENES -- "$B"/corpus/*.obj &
PID=$!
while kill -0 $PID 2>/dev/null; do
  RSS=$(awk '/VmRSS/ {print $2}' /proc/$PID/status 2>/dev/null || echo 0)
  if [ "${RSS:-0}" -gt 8000000 ]; then echo "sanitize: driver above 8 GB RSS, killed"; kill -9 $PID; exit 1; fi
  sleep 1
done
wait $PID
