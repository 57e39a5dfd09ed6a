"""Mixed-length batch (C5) on the GPU: every slide's output equals its own B = 1 forward."""
import pytest
import torch

import oracle as orc
from gigapath import batch

pytestmark = pytest.mark.gpu


def test_mixed_batch_equals_individual_forwards():
    from gigapath import slide_encoder
    cfg = orc.arch_config("gigapath_slide_enc12l768d")
    model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}, strict=True)
    model = model.cuda().eval()
    slides = []
    for i, n in enumerate([300, 2500, 1200, 5000]):
        x, c = orc.synthetic_slide(n, seed_x=10 + i, seed_c=20 + i)
        slides.append((torch.from_numpy(x[0]).cuda(), torch.from_numpy(c[0]).cuda()))
    out = batch.encode_slides(model, slides, all_layer_embed=True)
    with torch.no_grad():
        for (x, c), got in zip(slides, out):
            ref = model(x[None], c[None], all_layer_embed=True)
            assert len(got) == len(ref) == 13
            for g, r in zip(got, ref):
                assert torch.equal(g, r)


def test_mixed_batch_graph_replays_bit_exact():
    """use_hip_graphs: slides replayed as captured graphs (two slides sharing a shape, so one graph
    is replayed twice per batch) -- every output equals the eager B = 1 forward."""
    from gigapath import slide_encoder
    cfg = orc.arch_config("gigapath_slide_enc12l768d")
    model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}, strict=True)
    model = model.cuda().eval()
    sizes = [400, 2600, 1300, 400, 5100, 900]
    slides = []
    for i, n in enumerate(sizes):
        x, c = orc.synthetic_slide(n, seed_x=30 + i, seed_c=40 + i)
        slides.append((torch.from_numpy(x[0]).cuda(), torch.from_numpy(c[0]).cuda()))
    with torch.no_grad():
        ref = [torch.stack(model(x[None], c[None], all_layer_embed=True)) for x, c in slides]
    model.use_hip_graphs = True
    for _ in range(2):                                    # capture pass, then pure replays
        out = batch.encode_slides(model, slides, all_layer_embed=True)
        torch.cuda.synchronize()
        for got, want in zip(out, ref):
            assert torch.equal(torch.stack(got), want)
    assert len(model._graphs) == 5
