#!/usr/bin/env python3
"""Entry script with the reference's name and CLI (`train.py`); launched by
``torchrun`` / ``python -m distributed_pytorch_example_amd.launch`` /
``entrypoint.sh`` exactly like the reference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_pytorch_example_amd.train import main  # noqa: E402

if __name__ == "__main__":
    main()
