"""Concurrent HIP-graph replays on several streams (run with -m gpu).

Round 1 hung the GPU replaying different slides' graphs on 4 streams at once.  Cause established
from the code: every graph was captured on ONE side stream, and a captured hipBLASLt
GEMM bakes the workspace PyTorch keeps per (handle, stream) (ATen/cuda/CUDAContextLight.h,
cublaslt_handle_stream_to_workspace) -- so concurrent replays of different graphs shared one GEMM
workspace (the stream-K partial tiles and their flags) and, for equal shapes, one activation
workspace.  Now graphs, their capture side streams and the engine's activation workspaces are per
CALLER stream; this test replays four slides' graphs concurrently on four streams and requires every
output to equal the serial eager forward bit for bit.
"""
import pytest
import torch

import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_four_stream_concurrent_graph_replays_equal_eager():
    from gigapath import slide_encoder
    cfg = orc.arch_config("gigapath_slide_enc12l768d")
    model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}, strict=True)
    model = model.cuda().eval()
    sizes = [24000, 17000, 30000, 24000]          # two equal shapes: must not share activation buffers
    slides = []
    for i, n in enumerate(sizes):
        x, c = orc.synthetic_slide(n, seed_x=70 + i, seed_c=80 + i)
        slides.append((torch.from_numpy(x).cuda(), torch.from_numpy(c).cuda()))
    with torch.no_grad():
        ref = [torch.stack(model(x, c, all_layer_embed=True)) for x, c in slides]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in slides]
    model.use_hip_graphs, model.graph_min_uses = True, 1
    model.validate_positions = False            # no per-call host sync between the replays
    try:
        with torch.no_grad():
            for s, (x, c) in zip(streams, slides):       # capture, one graph per caller stream
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    model(x, c, all_layer_embed=True)
            torch.cuda.synchronize()
            assert len(model._graphs) == 4
            for _ in range(3):                            # concurrent replays
                outs = []
                for s, (x, c) in zip(streams, slides):
                    with torch.cuda.stream(s):
                        outs.append(torch.stack(model(x, c, all_layer_embed=True)))
                torch.cuda.synchronize()
                for i, (got, want) in enumerate(zip(outs, ref)):
                    assert torch.equal(got, want), i
        assert len(model._graphs) == 4
    finally:
        model.use_hip_graphs, model.graph_min_uses = False, 2
        model.validate_positions = True
        for k in list(model._graphs):
            model._drop_graph(k)
