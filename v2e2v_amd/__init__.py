"""v2e2v_amd -- MI355X-native (gfx950 HIP) CISTA-LSTC event-to-video hot path.

Drop-in for ``e2v.e2v_model.CistaLSTCNet`` of lsying009/V2E2V.
"""
from .e2v_model import CistaLSTCNet  # noqa: F401

__all__ = ["CistaLSTCNet"]
