source tools/gpu_steps.sh
export TMPDIR=/tmp
step gputests47 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke47 300 python -c "import __graft_entry__ as g; g.smoke()"
step ps47a 30 bash -c 'ps -eo pid,ppid,pcpu,etimes,rss,comm --sort=-pcpu | head -40; echo; ps -e --no-headers | wc -l; cat /proc/loadavg; ls /dev/shm | head; df -h /dev/shm /tmp | tail -2'
step b47_short1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step ps47b 30 bash -c 'ps -eo pid,ppid,pcpu,etimes,rss,comm --sort=-pcpu | head -20; cat /proc/loadavg'
step b47_short2 300 python bench.py --gpus 1 --steps 20 --warmup 5
