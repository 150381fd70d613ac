"""Runs bench.py's rank logic with every torchrun rank on GPU 0 (LOCAL_RANK
forced to 0): RCCL refuses two ranks on one GPU, so this exercises bench.py's
fallback -- node shards exchanging their lists through the host over gloo --
end to end on a one-GPU box.  Diagnostic / test aid, not the product path.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      --master-port P tools/bench_one_gpu_ranks.py --gpus 2 [bench args]
"""
import os
import runpy
import sys

os.environ["LOCAL_RANK"] = "0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
