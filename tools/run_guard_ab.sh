set -o pipefail
for v in base g0 g16 g32; do
  echo "== $v"
  CRIMP_LIB=build/variants/$v.so timeout -k 10 150 python3 -u tools/dbg_part.py 2>&1 | grep -v amdgpu.ids | grep -E "repeat identical|partition" || exit 1
  CRIMP_LIB=build/variants/$v.so timeout -k 10 150 python3 -u tools/dbg_2d.py 2>&1 | grep -v amdgpu.ids | grep -E "repeat|row|host" || exit 1
done
timeout -k 10 600 python3 -u tools/ab_search.py base g0 g16 g32 2>&1 | grep -v amdgpu.ids
