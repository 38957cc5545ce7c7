"""srsue_amd -- MI355X-native LTE downlink PDSCH receiver behind srsUE's srslte_ue_dl / srslte_pdsch API.

The product is the C-ABI library ``srsue_amd/libsrsue_amd.so`` (hand-written gfx950 HIP kernels +
host C++ planner), declared in ``include/srslte/srslte.h`` (per-TTI, srsLTE-1.0 compatible) and
``include/mi_dl.h`` (batched).  This package only binds it (``srsue_amd.abi``) for tests and the
benchmark; importing it does not touch the GPU.
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
