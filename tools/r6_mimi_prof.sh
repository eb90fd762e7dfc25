# config 5's context encode as the codec sees it (192 segments x 5 s), kernel trace + stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mprof -o run -- python3 tools/mimi_prof.py 192 5 > gpurun_out/mprof/out.txt 2> gpurun_out/mprof/err.txt || { tail -5 gpurun_out/mprof/err.txt; exit 1; }
cat gpurun_out/mprof/out.txt
python3 tools/kstats.py $(find gpurun_out/mprof -name "*kernel_stats.csv" | head -1) 30
