"""P2 on the MI355X: the product (HIP kernel through the C ABI, every kernel specialisation) against
16 independent runs of the reference binary itself, pinned in tests/golden/ref_fidelity_256x192_s256.npz
(tests/fidelity.py has the statistics and their calibration). The reference is not needed here.

P1 (bit-exact with the CPU contract) says the GPU computes the contract; this says the contract,
as the GPU runs it, estimates the same image as the reference (`smallpt.cpp:528-542`).
"""
import numpy as np
import pytest

import fidelity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kernel,est", [(k, e) for k in ("head", "const", "cornell", "generic")
                                        for e in ("nee", "cos")]
                         + [("generic", "uni"), ("auto", "q05"), ("generic", "q05"),
                            ("auto", "sph16"), ("generic", "sph16"), ("auto", "sph")])
def test_product_estimates_the_reference_image(spt, est, kernel):
    """uni: the uniform-hemisphere scattering (SPT_FLAG_UNIFORM_SCATTER, generic kernel) against the
    reference built with its commented-out uniform body (smallpt_uni_xs). q05: NEE-mix Q = 0.5
    (smallpt_q05_xs). sph / sph16: config 5's 32-sphere scene against the reference's own Sphere
    class (smallpt_sph_xs / smallpt_sph16_xs, depth cap 16): auto = the all-DIFF sphere kernel
    (TopoSphDiff)."""
    fx = fidelity.load_fixture()
    w, h, spp, k = fx["w"], fx["h"], fx["spp"], fx["k"]
    prims = fidelity.scene_of(spt, est)
    own = []
    for seed in range(1, 17):
        kw = fidelity.params_of(est)
        kw["flags"] = kw.get("flags", 0) | spt.kernel_flag(kernel)
        p = spt.default_params(width=w, height=h, spp=spp, seed=seed, **kw)
        img = spt.render(prims, spt.Camera(aspect=w / h), p)
        own.append(fidelity.blocks(img, k))
    zg, z2 = fidelity.compare(fx[est], own)
    assert np.all(np.abs(zg) < fidelity.GLOBAL_Z_MAX), zg
    assert z2 < fidelity.BLOCK_Z2_MAX, z2
