"""The bench's compaction leg alone with the library's host phase trace (SLATE_HOST_TRACE=1 on
stderr): where slate_compact's wall time goes (tooling)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]

if __name__ == "__main__":
    import torch  # noqa: F401  (torch first: see DESIGN §7, two HIP runtimes)
    import bench
    import slatecodec as sc
    ctx = sc.Context(0)
    kv = int(sys.argv[1]) if len(sys.argv) > 1 else 2_500_000
    print(json.dumps(bench.compaction_leg(sc, ctx, None, kv_per_sst=kv)))
