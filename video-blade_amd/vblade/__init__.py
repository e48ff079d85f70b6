"""vblade — MI355X-native adaptive block-sparse attention for Video-BLADE's video DiTs.

Drop-in for the reference's ``attn.inner_attention`` surface (CogVideoX-5B, Wan2.1-1.3B) and for
the external ``block_sparse_attn_func`` op; every hot-path byte is computed by hand-written HIP
kernels in ``libvblade_hip.so`` (C ABI: include/vblade.h).
"""
from ._lib import VBladeError, load as load_library  # noqa: F401
from .attention import (  # noqa: F401
    AdaptiveBlockSparseAttn,
    AdaptiveBlockSparseAttnTrain,
    GilbertRearranger,
    draw_sample_offsets,
    retain_counts,
)
from .autograd import adaptive_split_attention, block_sparse_attn_func  # noqa: F401
from .patch import (  # noqa: F401
    CogVideoXBlockSparseAttnProcessor,
    WanBlockSparseAttnProcessor,
    set_adaptive_block_sparse_attn_wanx,
    set_block_sparse_attn_cogvideox,
)

__version__ = "0.1.0"
