# Display-read rate of the window loop against the NUMA node its process runs
# on (measurement aid): the GPU's node, each node's CPUs, and dropin_rate's
# loop rate with the process bound to each node's CPUs.
set -e
for f in /sys/class/drm/card*/device/numa_node; do echo "$f: $(cat $f)"; done 2>/dev/null | head -4
for n in /sys/devices/system/node/node*; do echo "$(basename $n) cpus $(cat $n/cpulist)"; done
p=$(python3 -c "import sys; sys.path.insert(0, 'final-stage-path-tracer-2-0_amd'); import scenes; print(scenes.write('c4', '/tmp/fs_scenes/c4'))")
for n in /sys/devices/system/node/node*; do
  cpus=$(cat $n/cpulist | cut -d, -f1)
  for r in 1 2; do
    echo "$(basename $n) run $r: $(timeout -k 10 120 taskset -c $cpus ./examples/dropin_rate $p 1920 1080 256 | cut -c1-200)"
  done
done
for r in 1 2 3; do echo "unbound run $r: $(timeout -k 10 120 ./examples/dropin_rate $p 1920 1080 256 | cut -c1-200)"; done
