#!/bin/bash
# Build variants of the library with extra compile flags and time each with bench.py.
#   VARIANTS="NAME:FLAGS;NAME2:FLAGS2" bash tools/exp_variants.sh
# e.g. VARIANTS="base:;wpe3:-DAWE_WAVES_PER_EU=3"; a file tools/exp_src/NAME.hip replaces the
# kernel source for variant NAME (untracked scratch copies for A/B runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BATCH=${BATCH:-256}
IFS=';' read -ra VS <<< "${VARIANTS:-base:}"
for v in "${VS[@]}"; do
  name=${v%%:*}; flags=${v#*:}
  src=awebox_amd/csrc/awegpu.hip
  if [ -f "tools/exp_src/$name.hip" ]; then src="tools/exp_src/$name.hip"; fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Wno-unused-value \
      -Wno-unused-result -I awebox_amd/csrc $flags $src -o awebox_amd/libawegpu.so || exit 3
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --batch $BATCH --no-cpu-baseline \
      > gpurun_out/exp_$name.json 2> gpurun_out/exp_$name.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$name rc=$rc" >> gpurun_out/exp.log; exit $rc; fi
  python -c "import json;d=json.load(open('gpurun_out/exp_$name.json'));print('$name', '$flags', round(d['roofline']['kernel_ms'],4), round(d['value']))" >> gpurun_out/exp.log
done
cat gpurun_out/exp.log
