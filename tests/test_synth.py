"""Synthetic corpora (backuwup_amd/synth.py): host and HBM builders agree byte for byte."""


def test_device_corpus_builders_match_host():
    """The HBM-side C3/C4 builders used by bench.py produce the host corpora's bytes."""
    import numpy as np
    from backuwup_amd.synth import (small_files, small_files_table, splitmix_bytes, vm_image_variants,
                                    vm_image_variants_torch)
    d, o, l = vm_image_variants((1 << 20) + 3, 4, seed=2, n_indels=6, n_overwrites=3)
    t, o2, l2 = vm_image_variants_torch((1 << 20) + 3, 4, "cpu", seed=2, n_indels=6, n_overwrites=3)
    assert np.array_equal(o, o2) and np.array_equal(l, l2)
    assert np.array_equal(t.numpy(), d)
    d, o, l = small_files(300, seed=4)
    u, o2, l2 = small_files_table(300, seed=4)
    blob = splitmix_bytes(4, u)
    assert np.array_equal(l, l2)
    for i in range(300):
        assert np.array_equal(d[int(o[i]):int(o[i] + l[i])], blob[int(o2[i]):int(o2[i] + l2[i])])
