"""CPU checks of the GPU tests' constructed cases (tests/render_cases.py)."""
from tests.render_cases import near_threshold_records


def test_needle_threshold_records_have_teeth():
    """The near-threshold records below are a real test of contraction-off: on some of them either FMA contraction
    of rec_needle's expression decides differently from the separately rounded one (CPU, numpy + exact rationals)."""
    _, dec = near_threshold_records()
    assert dec[:, 0].any() and not dec[:, 0].all()
    assert (dec[:, 0] != dec[:, 1]).sum() >= 10 and (dec[:, 0] != dec[:, 2]).sum() >= 10
