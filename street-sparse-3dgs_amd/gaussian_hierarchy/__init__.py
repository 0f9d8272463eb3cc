"""Drop-in for the reference's `gaussian_hierarchy` extension (the un-vendored
submodules/gaussianhierarchy): the LOD-cut entry points its render / train scripts import,
    from gaussian_hierarchy._C import expand_to_size, get_interpolation_weights
(render_hierarchy.py:27, train_post.py, render_hierarchy_final.py:19, render_position.py:11),
computed by the gfx950 kernels of libgsr_hip.so (csrc/lod.hip)."""
from . import _C  # noqa: F401
