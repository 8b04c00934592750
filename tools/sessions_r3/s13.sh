source tools/gpu_steps.sh
step numa 10 bash -c 'cat /sys/fs/cgroup/cpu.stat; ls /sys/devices/system/node/ | grep node; for n in /sys/devices/system/node/node*; do echo $n $(cat $n/cpulist); done; lscpu | grep -i "model name\|L3\|NUMA\|Socket"'
for i in 1 2; do
  step aff0_$i 300 python tools/probe/affinity_ab.py --cpus 0 -- --gpus 1 --steps 20 --warmup 5
  step aff16_$i 300 python tools/probe/affinity_ab.py --cpus 16 -- --gpus 1 --steps 20 --warmup 5
  step aff24_$i 300 python tools/probe/affinity_ab.py --cpus 24 -- --gpus 1 --steps 20 --warmup 5
done
step aff0_long 300 python tools/probe/affinity_ab.py --cpus 0 -- --gpus 1
step aff16_long 300 python tools/probe/affinity_ab.py --cpus 16 -- --gpus 1
