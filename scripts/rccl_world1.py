"""RCCL plumbing check on one GPU: the multi-GPU bench path (distributed.run_sharded: nccl process group,
collectives on the engine stream through torch.cuda.ExternalStream) at world size 1, in both modes.
(RCCL refuses two ranks on one device, so this is as far as a one-GPU box goes.)"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
from visual_inertial_bundle_adjustment_amd.distributed import run_sharded  # noqa: E402

a = argparse.Namespace(config=sys.argv[1] if len(sys.argv) > 1 else "B", steps=3, warmup=1, no_cpu_baseline=True,
                       precision="fp64", rs_tables="device")
run_sharded(a, 0, 1, 0)
