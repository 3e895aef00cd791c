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


def test_c5_ranks_split_families():
    """bench.py's C5 layout: ranks 2f and 2f+1 hold files 0-7 and 8-15 of family f (base seed
    1 + f), rebased to their own buffers; the pair together is the family's 16-file corpus."""
    import numpy as np
    import torch
    import bench
    from backuwup_amd.synth import vm_image_variants
    gib = (1 << 20) / float(1 << 30)
    for fam in (0, 1):
        d, o, l = vm_image_variants(1 << 20, 16, seed=1 + fam)
        for half in (0, 1):
            t, o2, l2, desc = bench.make_workload("c5", gib, 2 * fam + half, torch.device("cpu"), 0)
            assert len(o2) == 8 and int(o2[0]) == 0 and int(o2[-1] + l2[-1]) == t.numel()
            assert np.array_equal(l2, l[8 * half:8 * half + 8])
            lo = int(o[8 * half])
            assert np.array_equal(t.numpy(), d[lo:lo + t.numel()])
            assert "family %d" % fam in desc
