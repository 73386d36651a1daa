set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2n
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --max-num-seqs 448 > gpurun_out/s2n/q49_s448.json 2> gpurun_out/s2n/q49_s448.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2n/q49_s384.json 2> gpurun_out/s2n/q49_s384.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --max-num-seqs 416 > gpurun_out/s2n/q49_s416.json 2> gpurun_out/s2n/q49_s416.err
