# The window loop (examples/dropin_rate) of an A/B build under a kernel + copy
# trace, for per-frame timelines (tools/frame_periods.py).
# usage: bash tools/prof_dropin256.sh TAG LIB SCENE FRAMES
set -e
tag=$1; lib=$2; sc=$3; n=$4
d=/tmp/fs_ablib_${lib%.so}; mkdir -p $d
cp final-stage-path-tracer-2-0_amd/$lib $d/libfsgpu.so
cp final-stage-path-tracer-2-0_amd/libfshost.so $d/
p=$(python3 -c "import sys; sys.path.insert(0, 'final-stage-path-tracer-2-0_amd'); import scenes; print(scenes.write('$sc', '/tmp/fs_scenes/$sc'))")
out=gpurun_out/$tag/${sc}_${lib%.so}
mkdir -p $out
LD_LIBRARY_PATH=$d timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out -o trace -- \
  ./examples/dropin_rate $p 1920 1080 $n > $out/run.json 2> $out/run.err
cat $out/run.json
