"""Host logic of the window attention op (gdino_amd/wattn.py): when the
kernel is handed NULL for rel_index (the kernel then computes the reference's
index, swin_transformer.py:104-115) and NULL for the shift mask (the kernel
computes the reference's region mask, :402-426).  CPU only: no kernel runs."""
import torch

from gdino_amd import wattn
from models.GroundingDINO.backbone.swin_transformer import relative_position_index, shifted_window_mask


def test_reference_index_is_passed_as_null_and_others_as_tensors():
    r = relative_position_index(7, 7)
    assert wattn._kernel_index(r.view(-1), 49) is None
    odd = (r.view(-1) * 7 + 3) % 169
    assert torch.equal(wattn._kernel_index(odd, 49), odd)
    assert wattn._kernel_index(relative_position_index(12, 12).view(-1), 144) is None


def test_index_check_follows_in_place_updates_and_never_trusts_a_reused_address():
    r = relative_position_index(7, 7)
    assert wattn._kernel_index(r.view(-1), 49) is None
    r[0, 1] = 5  # in-place change (a checkpoint load would do this): re-checked
    assert wattn._kernel_index(r.view(-1), 49) is not None
    # a new tensor at a possibly reused address is a new object: re-checked
    for _ in range(3):
        t = ((relative_position_index(7, 7) + 1) % 169).view(-1)
        assert wattn._kernel_index(t, 49) is not None
        del t


def test_region_mask_is_recognised_by_geometry():
    m = shifted_window_mask(21, 35, 7, 3, "cpu")
    assert wattn._is_region_mask(m, (19, 30), 7, 3)
    assert not wattn._is_region_mask(m, (19, 30), 7, 2)
    assert not wattn._is_region_mask(m.clone(), (19, 30), 7, 3)  # an arbitrary tensor is read as given
