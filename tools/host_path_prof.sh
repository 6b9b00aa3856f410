# Kernel + copy trace of the host path loop (tools/host_path_trace.py); read with tools/timeline.py gpurun_out/hp
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hp -o run -- python3 tools/host_path_trace.py > gpurun_out/hp.log 2>&1
