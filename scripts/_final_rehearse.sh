set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r5r_reh
timeout -k 10 500 python -u scripts/camera_rehearse.py --frames 10 --out gpurun_out/r5r_reh/r5_rehearse.json > gpurun_out/r5r_reh/r5_rehearse.log 2>&1
timeout -k 10 600 python -u scripts/camera_rehearse.py --frames 10 --shader ao --modes view close --out gpurun_out/r5r_reh/r5_rehearse_ao.json > gpurun_out/r5r_reh/r5_rehearse_ao.log 2>&1
