"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import hashlib

import numpy as np
import pytest
import torch

import oracle as orc
from conftest import load_golden


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


CFG = orc.arch_config("gigapath_slide_enc12l768d")


def test_param_count_and_keys(golden_meta):
    keys = orc.state_dict_keys(CFG)
    assert [[k, list(s)] for k, s in keys] == golden_meta["state_dict"]
    assert len(keys) == 247
    n = sum(int(np.prod(s)) for _, s in keys)
    assert n == golden_meta["n_params"] == 86330880          # demo/run_gigapath.ipynb cell 9
    assert golden_meta["n_params_longnet"] == 85148160


def test_weights_generator_stable(golden_meta):
    W = orc.make_weights(CFG, seed=0, perturb=True)
    assert orc.weights_sha256(W) == golden_meta["weights_sha256"]


def test_segment_schedules(golden_meta):
    for mw, segs in golden_meta["schedules"].items():
        assert orc.segment_schedule(int(mw), 256) == segs
    assert golden_meta["schedules"]["262144"] == [1024, 5792, 32768, 185363, 1048576]


def test_pos_table_rows_bit_exact(golden_meta):
    assert golden_meta["pos_table_bit_exact"]
    g = load_golden("pos_embed_rows.npz")
    tab = orc.sincos_axis_table(768, 1000)
    ours = orc.pos_embed_rows(g["rows"], tab, 1000)
    assert np.array_equal(ours.view(np.uint32), g["values"].view(np.uint32))


def test_coords_to_pos_bit_exact():
    g = load_golden("coords_to_pos.npz")
    assert np.array_equal(orc.coords_to_pos(g["coords"], 1000, 256), g["pos"])


def test_pos_index_errors():
    tab = orc.sincos_axis_table(768, 1000)
    with pytest.raises(IndexError):
        orc.pos_embed_rows(np.array([1000001]), tab, 1000)
    # negative indices wrap like torch indexing
    r = orc.pos_embed_rows(np.array([-1]), tab, 1000)
    assert np.array_equal(r, orc.pos_embed_rows(np.array([1000000]), tab, 1000))


def test_index_maps_against_reference(golden_meta):
    small = load_golden("index_maps_small.npz")
    for ent in golden_meta["index_maps"]:
        L = ent["L"]
        for b, (sl, r) in enumerate(zip(ent["segs"], ent["ratios"])):
            tok = orc.gather_index(L, sl, r, 16)
            n_idx, i_idx = orc.scatter_index(L, sl, r, 16)
            assert sha(tok) == ent["sha256"]["gather_%d" % b], (ent["tag"], L, b)
            assert sha(n_idx) == ent["sha256"]["scatter_n_%d" % b], (ent["tag"], L, b)
            assert sha(i_idx) == ent["sha256"]["scatter_i_%d" % b], (ent["tag"], L, b)
            key = "%s_%d_gather_%d" % (ent["tag"], L, b)
            if key in small:
                assert np.array_equal(small[key], tok)


def test_misaligned_schedule_is_exercised(golden_meta):
    """wsi250000 @ L=30001: 23170 % 4 != 0 with 2 segments -> the reference's shifted scatter."""
    ent = [e for e in golden_meta["index_maps"] if e["tag"] == "wsi250000"][0]
    geo = orc.branch_geometry(ent["L"], ent["segs"][2], ent["ratios"][2], 16)
    assert geo["nseg"] == 2 and geo["g"] != geo["s"]


def test_dilated_attention_module_golden():
    g = load_golden("dilated_attention_custom.npz")
    W = {k: torch.from_numpy(v) for k, v in orc.make_weights(CFG, seed=0).items()}
    y = orc.dilated_attention(torch.from_numpy(g["x"]), W, "encoder.layers.0.self_attn",
                              list(g["segs"]), list(g["ratios"]), 16)
    np.testing.assert_allclose(y.numpy(), g["y"], rtol=0, atol=2e-5 * np.abs(g["y"]).max())


@pytest.mark.parametrize("N,B", [(1024, 1), (4097, 1), (600, 2)])
def test_end_to_end_golden(N, B, golden_meta):
    g = load_golden("e2e_N%d_B%d.npz" % (N, B))
    W = {k: torch.from_numpy(v) for k, v in orc.make_weights(CFG, seed=0).items()}
    x, coords = orc.synthetic_slide(N, B=B)
    ent = [e for e in golden_meta["e2e"] if e["N"] == N and e["B"] == B][0]
    assert sha(x) == ent["x_sha256"] and sha(coords) == ent["coords_sha256"]
    torch.set_num_threads(min(8, torch.get_num_threads()))
    with torch.no_grad():
        allv = torch.stack(orc.slide_encoder_forward(W, x, coords, CFG, all_layer_embed=True)).numpy()
        last = orc.slide_encoder_forward(W, x, coords, CFG)[0].numpy()
        gp = orc.slide_encoder_forward(W, x, coords, CFG, global_pool=True)[0].numpy()
    tol = 1e-4
    np.testing.assert_allclose(allv, g["all_layer"], rtol=0, atol=tol * np.abs(g["all_layer"]).max())
    np.testing.assert_allclose(last, g["last"], rtol=0, atol=tol * np.abs(g["last"]).max())
    np.testing.assert_allclose(gp, g["gp_last"], rtol=0, atol=tol * np.abs(g["gp_last"]).max())


def test_end_to_end_golden_c2_16k(golden_meta):
    """The oracle at config C2's size (16,384 tiles, multi-segment branches 0-1) against the
    reference's own fp32 output: one all_layer_embed forward (~40 s on 8 threads)."""
    N = 16384
    g = load_golden("e2e_N%d_B1.npz" % N)
    W = {k: torch.from_numpy(v) for k, v in orc.make_weights(CFG, seed=0).items()}
    x, coords = orc.synthetic_slide(N)
    ent = [e for e in golden_meta["e2e"] if e["N"] == N and e["B"] == 1][0]
    assert sha(x) == ent["x_sha256"] and sha(coords) == ent["coords_sha256"]
    torch.set_num_threads(min(8, torch.get_num_threads()))
    with torch.no_grad():
        allv = torch.stack(orc.slide_encoder_forward(W, x, coords, CFG, all_layer_embed=True)).numpy()
    np.testing.assert_allclose(allv, g["all_layer"], rtol=0, atol=1e-4 * np.abs(g["all_layer"]).max())


def test_tiny_slides_golden(golden_meta):
    """The oracle on the tiny / ragged slides (N = 1, 2, 31, 255, 257, 1023 and 3 x 5 tiles) against the
    reference's own fp32 outputs (tests/golden/tiny_slides.npz, make_golden.py --tiny), which also hold the
    reference's bf16 run that pins the GPU tests' tolerance there (test_gpu_model.check_tiny)."""
    g = load_golden("tiny_slides.npz")
    W = orc.make_weights(CFG, seed=0)
    assert orc.weights_sha256(W) == golden_meta["tiny"]["weights_sha256"]
    Wt = {k: torch.from_numpy(v) for k, v in W.items()}
    torch.set_num_threads(min(8, torch.get_num_threads()))
    for ent in golden_meta["tiny"]["cases"]:
        N, B = ent["N"], ent["B"]
        if N > 300:                 # (N = 1023: ~1 min of oracle on the CPU; the GPU test still uses it)
            continue
        x, coords = orc.synthetic_slide(N, B=B)
        assert sha(x) == ent["x_sha256"] and sha(coords) == ent["coords_sha256"]
        with torch.no_grad():
            allv = torch.stack(orc.slide_encoder_forward(Wt, x, coords, CFG, all_layer_embed=True)).numpy()
        ref = g["N%d_B%d_fp32" % (N, B)]
        np.testing.assert_allclose(allv, ref, rtol=0, atol=1e-4 * np.abs(ref).max())
        # the recorded deviation is what the bf16 fixture shows, vector by vector
        bf = g["N%d_B%d_bf16" % (N, B)]
        vec = max(float(np.abs(bf[i] - ref[i]).max() / np.abs(ref[i]).max()) for i in np.ndindex(*ref.shape[:-1]))
        assert vec == pytest.approx(ent["ref_bf16_rel_vec_max"], rel=1e-6)
