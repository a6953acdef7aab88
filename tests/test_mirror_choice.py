"""Which device-decode paths ``h2d`` puts through the HBM log mirror (DeviceLoader._mirror): only
an explicit 'dma'.  'auto' stays zero-copy: the mirror still collapses on some runs
(profiles/r03_final/c4_auto_mirror_trial/)."""
import pytest

from torchkafka_amd.loader.device_loader import DeviceLoader


def _loader(h2d, device_decode=True):
    L = object.__new__(DeviceLoader)
    L.h2d = h2d
    L._device_decode = lambda: device_decode
    return L


@pytest.mark.parametrize("h2d,dd,want", [
    ("dma", True, True),          # opt-in: any device decode
    ("dma", False, False),        # nothing read from the logs
    ("auto", True, False),        # the default stays zero-copy
    ("zerocopy", True, False),
])
def test_mirror_choice(h2d, dd, want):
    assert _loader(h2d, dd)._mirror() is want
