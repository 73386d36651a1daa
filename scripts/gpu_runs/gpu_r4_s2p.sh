set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2p
MXS_PF_ATTN_DMA=1 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "paged_prefill or prefill_softmax" > gpurun_out/s2p/kt_dma.log 2>&1 || true
grep -cE "PASSED" gpurun_out/s2p/kt_dma.log || true
grep -E "FAILED|Error" gpurun_out/s2p/kt_dma.log | head -20 || true
timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/s2p/reg.jsonl 2>&1
MXS_PF_ATTN_DMA=1 timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/s2p/dma.jsonl 2>&1
timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/s2p/reg2.jsonl 2>&1
MXS_PF_ATTN_DMA=1 timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/s2p/dma2.jsonl 2>&1
for f in reg dma reg2 dma2; do echo $f; grep "{" gpurun_out/s2p/$f.jsonl; done
