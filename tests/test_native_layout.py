"""Host-side launch layouts of the native extension that need no GPU: the LeNet-5 images-per-workgroup
policy (csrc/lenet_fused.hip lenet_ipw / lenet_blocks) and the irregular-geometry routing of the conv
dispatch (csrc/bindings.cpp set_conv_geom: only the generic implicit GEMM takes it)."""
import pytest

from distriflow_amd import native, ops

m = native.get(build_if_missing=False)
pytestmark = pytest.mark.skipif(m is None, reason="native extension not built")


@pytest.mark.parametrize("B,ipw", [(1, 1), (32, 1), (256, 1), (257, 2), (512, 2), (513, 4), (1024, 4),
                                   (1025, 8), (2048, 8), (2049, 8), (4096, 8), (8192, 8)])
def test_lenet_images_per_workgroup(B, ipw):
    """One workgroup per CU (256) with the fewest images per workgroup, else 8 (the full-batch kernel)."""
    assert ops.lenet_blocks(B) == -(-B // ipw)


def test_irregular_conv_geometry_refuses_specialised_paths():
    """A regular 3x3 / stride 1 / pad 1 64-channel conv may accumulate BatchNorm sums in the specialised
    kernels' epilogues in both directions; the same conv with asymmetric padding, a (2, 1) stride or a 3x5
    kernel runs on the generic kernel, whose epilogue takes the forward sums only (mode 0)."""
    B, H, W, C, N = 4, 16, 16, 64, 64

    def ok(KH, KW, stride, pad, OH, OW, dgrad):
        Kp = -(-(KH * KW * (N if dgrad else C)) // 32) * 32
        return ops.conv_bacc_ok(B, H, W, C, OH, OW, N, KH, KW, stride, pad, Kp, dgrad=dgrad, mode=1 if dgrad else 0,
                                has_mask=dgrad)

    assert ok(3, 3, 1, 1, 16, 16, True)
    assert not ok(3, 3, 2, (0, 0), 8, 8, True)          # odd 'same' total: pad 0 top / left, 1 bottom / right
    assert not ok(3, 3, (2, 1), (1, 1), 8, 16, True)
    assert not ok(3, 5, 1, (1, 2), 16, 16, True)
    assert ok(3, 5, 1, (1, 2), 16, 16, False)            # generic forward: epilogue sums, mode 0
