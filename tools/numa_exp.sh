set -u
O=gpurun_out/r06n; mkdir -p $O
(lscpu | grep -i numa; for f in /sys/class/drm/card*/device/numa_node; do echo $f $(cat $f); done; cat /proc/loadavg) > $O/numa.txt 2>&1
N0=$(lscpu | grep "NUMA node0 CPU" | awk '{print $NF}')
N1=$(lscpu | grep "NUMA node1 CPU" | awk '{print $NF}')
echo "node0 $N0 node1 $N1" >> $O/numa.txt
for cfg in none node0 node1 none; do
  case $cfg in none) P="";; node0) P="taskset -c $N0";; node1) P="taskset -c $N1";; esac
  echo "== $cfg" >> $O/sweep.jsonl
  timeout -k 10 300 $P python -u tools/xdp_host_sweep.py --threads 16 --chunks 524288 --per-call 65536,1048576 >> $O/sweep.jsonl 2>> $O/sweep.err || exit $?
done
cat $O/numa.txt; cat $O/sweep.jsonl
