"""``python -m flink_ml_amd.bench.run <config.json> [--output-file out.json] [--pattern REGEX]``
(the reference's ``benchmark-run.sh``). Multi-GPU: launch with ``torch.distributed.run``."""
import sys

from .runner import main

if __name__ == "__main__":
    sys.exit(main())
