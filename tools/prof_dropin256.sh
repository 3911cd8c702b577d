set -e
p=$(python3 -c "import sys; sys.path.insert(0, 'final-stage-path-tracer-2-0_amd'); import scenes; print(scenes.write('c4', '/tmp/fs_scenes/c4'))")
mkdir -p gpurun_out/r06stall
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06stall/prof -o trace -- ./examples/dropin_rate $p 1920 1080 256 > gpurun_out/r06stall/run.json 2> gpurun_out/r06stall/run.err
cat gpurun_out/r06stall/run.json
