"""Worker script for tests/test_dist.py::test_launcher_*: records the torchrun-style environment
bench.launch_workers gives each rank (test infrastructure)."""
import json
import os
import sys

out_dir, fail_rank = sys.argv[1], int(sys.argv[2])
env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
with open(os.path.join(out_dir, f"rank{env['RANK']}.json"), "w") as f:
    json.dump(env, f)
sys.exit(3 if int(env["RANK"]) == fail_rank else 0)
