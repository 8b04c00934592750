#!/bin/bash
# Clock of this job's CPUs (cpuset) while idle and while bench.py runs:
# samples scaling_cur_freq every 50 ms into gpurun_out/cpufreq.log.
#   bash tools/probe/cpufreq_probe.sh [bench args...]
mkdir -p gpurun_out
cpus=$(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null || cat /proc/self/status | awk '/Cpus_allowed_list/{print $2}')
echo "cpuset: $cpus" > gpurun_out/cpufreq.log
ls /sys/devices/system/cpu/cpu0/cpufreq/ >> gpurun_out/cpufreq.log 2>&1
cat /sys/devices/system/cpu/cpu0/cpufreq/scaling_governor >> gpurun_out/cpufreq.log 2>&1
list=$(python3 -c "
import sys
s='$cpus'; out=[]
for part in s.split(','):
    if '-' in part:
        a,b=part.split('-'); out+=range(int(a),int(b)+1)
    elif part: out.append(int(part))
print(' '.join(map(str,out)))")
sample() {
  while true; do
    line="$(date +%s.%N)"
    for c in $list; do line="$line $(cat /sys/devices/system/cpu/cpu$c/cpufreq/scaling_cur_freq 2>/dev/null || echo -)"; done
    echo "$line" >> gpurun_out/cpufreq.log
    sleep 0.05
  done
}
sample &
S=$!
sleep 1
echo "bench start $(date +%s.%N)" >> gpurun_out/cpufreq.log
timeout -k 10 240 python bench.py "$@" > gpurun_out/cpufreq_bench.log 2>&1
rc=$?
echo "bench end $(date +%s.%N) rc=$rc" >> gpurun_out/cpufreq.log
sleep 1
kill $S
exit $rc
