set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
run() {  # $1 tag, rest env
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u scripts/probe.py --config c2 --warmup 3 --steps 64 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "$tag failed"; tail -20 gpurun_out/ab_$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', round(d['gpu']['default']['gpu_it_per_s'],1))"
}
run cur4 MILP_HOST_THREADS=4 && run v5_4 MI_LP_LIB=$R/or-tools_amd/lib/libmi_lp_v5.so MILP_HOST_THREADS=4 && run cur1 MILP_HOST_THREADS=1 && run v5_1 MI_LP_LIB=$R/or-tools_amd/lib/libmi_lp_v5.so MILP_HOST_THREADS=1 && run cur4b MILP_HOST_THREADS=4 && nproc && cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -E "Model name|^CPU\(s\)|Thread" | head -4
