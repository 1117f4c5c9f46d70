echo "nproc=$(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/cgroup; 
lscpu | grep -E "Model name|Socket|Core|Thread|NUMA node|L3" 
env | grep -E "OMP|MAX_JOBS|HIP|ROCR|CUDA" 
cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null
