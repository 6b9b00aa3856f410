export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --output-format csv -d gpurun_out/hp -o run -- python3 tools/host_path_trace.py > gpurun_out/hp.log 2>&1
