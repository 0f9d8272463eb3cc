"""Drop-in for the reference's `simple_knn` extension (submodules/simple-knn): `from
simple_knn._C import distCUDA2` (scene/gaussian_model.py:20,207) resolves here, on the gfx950
kernel csrc/knn.hip."""
