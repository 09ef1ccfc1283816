"""Multi-process launcher (reference: /root/reference/launch.py), fail-fast version.

    python launch.py --nproc_per_node=8 -m main parameter.epochs=200
"""
from simclr_amd.runtime.launcher import main

if __name__ == "__main__":
    main()
