"""RCCL (torch 'nccl' backend) lockstep on one GPU -- runs last in the GPU session."""
import pytest

pytestmark = pytest.mark.gpu


def test_lockstep_rccl_world1():
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import nccl_probe

    nccl_probe.main()
