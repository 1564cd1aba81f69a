# Host sanitizers (CPU only; GPU AddressSanitizer is not available on the
# pool): the product's host C++ (slio_ikf.cpp, slio_imu.cpp, slio_s2m.cpp)
# and the CPU oracle built with AddressSanitizer + UndefinedBehaviorSanitizer
# (clang, one runtime in the process), then the CPU test suite against them.
# The product's device objects are the in-tree build's (_obj, no sanitizer:
# -fsanitize goes to the host side only).  Log: profiles/r06_sanitizers.log
set -e -o pipefail
cd "$(dirname "$0")/.."
python3 -c "from agi_lidar_slam_amd import build; build.build()"
tag=$(python3 -c "from agi_lidar_slam_amd import build; print(build.source_hash())")
out=_var/san
mkdir -p $out
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=undefined"
F="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -DSLIO_SOURCE_HASH=\"$tag\" -Iinclude"
for s in slio_ikf.cpp slio_imu.cpp slio_s2m.cpp; do
  /opt/rocm/bin/hipcc $F $SAN -c agi_lidar_slam_amd/csrc/$s -o $out/$s.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -fsanitize=address,undefined -shared-libsan \
  agi_lidar_slam_amd/_obj/slio_device.hip.o agi_lidar_slam_amd/_obj/slio_lio.hip.o $out/*.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o $out/libslio_san.so
CLANG=/opt/rocm/lib/llvm/bin/clang++
$CLANG -O1 -g -std=c++17 -fPIC -fopenmp -ffp-contract=off -fno-fast-math -fsanitize=address,undefined \
  -fno-sanitize-recover=undefined -fno-omit-frame-pointer -shared-libsan -shared \
  oracle/slio_oracle.cpp oracle/frontend_oracle.cpp oracle/map_oracle.cpp oracle/imu_oracle.cpp \
  oracle/lio_s2m_oracle.cpp -o $out/libslio_oracle_san.so
RT=$($CLANG -print-file-name=libclang_rt.asan-x86_64.so)
echo "runtime $RT"
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:allocator_may_return_null=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  SLIO_SANITIZE_LIB=$out/libslio_san.so SLIO_ORACLE_LIB=$out/libslio_oracle_san.so \
  timeout 1800 python3 -m pytest tests -m "not gpu" -x -q -p no:cacheprovider 2>&1 | tee profiles/r06_sanitizers.log
