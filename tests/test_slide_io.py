"""Slide-file input formats (gigapath/slide_io.py; reference finetune/datasets/slide_datatset.py:148-193).

HDF5 parity is pinned against files built from the format specification by tests/h5_spec_writer.py
(h5py is absent from this image; no HDF5 file ships with the reference or the image).  When h5py is
importable the last test also cross-checks against it.
"""
import os

import numpy as np
import pytest
import torch

from gigapath import slide_io
from h5_spec_writer import Writer


def _slide(n=57, dim=24, seed=0, dtype=np.float32):
    rng = np.random.default_rng(seed)
    feats = rng.standard_normal((n, dim)).astype(dtype)
    coords = (rng.integers(0, 400, size=(n, 2)) * 256).astype(np.int64)
    return feats, coords


ATTRS = {"patch_size": np.float64(256.0), "levels": np.arange(3, dtype=np.int32), "name": "slide-0001 µm",
         "tag": np.bytes_(b"abc"), "is_tumor": True}


def _check_attrs(got):
    assert got["patch_size"] == 256.0 and isinstance(got["patch_size"], np.floating)
    np.testing.assert_array_equal(got["levels"], np.arange(3))
    assert got["levels"].dtype == np.int32
    assert got["name"] == "slide-0001 µm"
    assert got["tag"] == b"abc"
    assert got["is_tumor"] is True or got["is_tumor"] == np.bool_(True)


@pytest.mark.parametrize("style,userblock,continuation", [("earliest", 0, False), ("earliest", 512, True),
                                                          ("latest", 0, False), ("latest", 1024, True)])
def test_contiguous_datasets_and_attrs(tmp_path, style, userblock, continuation):
    feats, coords = _slide()
    w = Writer(style, userblock=userblock, continuation=continuation)
    w.dataset("features", feats, attrs=ATTRS)
    w.dataset("coords", coords)
    p = str(tmp_path / "s.h5")
    w.save(p)
    assets, attrs = slide_io.read_assets_from_h5(p)
    assert sorted(assets) == ["coords", "features"]
    np.testing.assert_array_equal(assets["features"], feats)
    np.testing.assert_array_equal(assets["coords"], coords)
    assert assets["features"].dtype == np.float32 and assets["coords"].dtype == np.int64
    _check_attrs(attrs["features"])
    assert attrs["coords"] == {}


@pytest.mark.parametrize("style", ["earliest", "latest"])
@pytest.mark.parametrize("filters", [(), ("deflate",), ("shuffle", "deflate"), ("shuffle", "deflate", "fletcher32")])
def test_chunked_filtered(tmp_path, style, filters):
    feats, coords = _slide(n=101, dim=40, seed=1, dtype=np.float16)
    w = Writer(style)
    # ragged edge chunks in both dims; leaf_max=4 forces a two-level chunk B-tree
    w.dataset("features", feats, layout="chunked", chunks=(16, 24), filters=filters, btree_leaf=4)
    w.dataset("coords", coords.astype(np.float32), layout="chunked", chunks=(32, 2), filters=filters)
    p = str(tmp_path / "c.h5")
    w.save(p)
    assets, _ = slide_io.read_assets_from_h5(p)
    np.testing.assert_array_equal(assets["features"], feats)
    np.testing.assert_array_equal(assets["coords"], coords.astype(np.float32))


@pytest.mark.parametrize("style", ["earliest", "latest"])
@pytest.mark.parametrize("rows,alloc_seed", [(1, None), (1, 3), (16, None), (16, 4)])
def test_row_slab_chunks(tmp_path, style, rows, alloc_seed):
    """CLAM-style feature files: chunks of whole rows (one tile per chunk), unfiltered, possibly laid
    out in the file out of row order -- read by runs of file-consecutive chunks."""
    feats, coords = _slide(n=203, dim=20, seed=2)
    w = Writer(style)
    w.dataset("features", feats, layout="chunked", chunks=(rows, 20), btree_leaf=64, alloc_seed=alloc_seed)
    w.dataset("coords", coords, layout="chunked", chunks=(rows, 2), alloc_seed=alloc_seed)
    w.dataset("be", feats.astype(">f8"), layout="chunked", chunks=(rows, 20))
    p = str(tmp_path / "r.h5")
    w.save(p)
    a, _ = slide_io.read_assets_from_h5(p)
    np.testing.assert_array_equal(a["features"], feats)
    np.testing.assert_array_equal(a["coords"], coords)
    np.testing.assert_array_equal(a["be"], feats.astype(np.float64))
    assert a["be"].dtype.isnative


def test_compact_and_big_endian(tmp_path):
    w = Writer("earliest")
    w.dataset("small", np.arange(6, dtype=np.int16).reshape(2, 3), layout="compact")
    w.dataset("be", np.arange(5, dtype=">f4") * 1.5)
    w.dataset("scalar", np.array(7, dtype=np.uint8))
    p = str(tmp_path / "m.h5")
    w.save(p)
    a, _ = slide_io.read_assets_from_h5(p)
    np.testing.assert_array_equal(a["small"], np.arange(6).reshape(2, 3))
    np.testing.assert_array_equal(a["be"], np.arange(5) * 1.5)
    assert a["be"].dtype == np.float32 and a["be"].dtype.isnative
    assert a["scalar"].shape == () and int(a["scalar"]) == 7


def test_get_images_from_path_h5(tmp_path):
    feats, coords = _slide(n=50)
    w = Writer()
    w.dataset("features", feats)
    w.dataset("coords", coords)
    p = str(tmp_path / "slide.h5")
    w.save(p)
    d = slide_io.get_images_from_path(p, max_tiles=30)
    assert d["img_lens"] == 30 and d["pad_mask"] == 0
    torch.testing.assert_close(d["imgs"], torch.from_numpy(feats[:30]))
    torch.testing.assert_close(d["coords"], torch.from_numpy(coords[:30]))
    g = torch.Generator().manual_seed(5)
    d = slide_io.get_images_from_path(p, max_tiles=1000, shuffle_tiles=True, generator=g)
    perm = torch.randperm(50, generator=torch.Generator().manual_seed(5))
    torch.testing.assert_close(d["imgs"], torch.from_numpy(feats)[perm])
    torch.testing.assert_close(d["coords"], torch.from_numpy(coords)[perm])   # tiles and coords stay paired


def test_get_images_from_path_pt_and_errors(tmp_path):
    x = torch.randn(12, 1536)
    p = str(tmp_path / "tiles.pt")
    torch.save(x, p)
    d = slide_io.get_images_from_path(p)
    torch.testing.assert_close(d["imgs"], x)
    assert d["coords"] == 0 and d["img_lens"] == 12
    with pytest.raises(ValueError):
        slide_io.get_images_from_path(str(tmp_path / "x.tiff"))
    w = Writer()
    w.dataset("features", np.zeros((3, 4), np.float32))
    q = str(tmp_path / "nocoords.h5")
    w.save(q)
    with pytest.raises(KeyError, match="coords"):
        slide_io.get_images_from_path(q)
    bad = tmp_path / "bad.h5"
    bad.write_bytes(b"not an hdf5 file at all" * 10)
    with pytest.raises(ValueError, match="superblock"):
        slide_io.read_assets_from_h5(str(bad))


def test_unsupported_filter_raises(tmp_path):
    w = Writer("earliest")
    w.dataset("features", np.zeros((8, 4), np.float32), layout="chunked", chunks=(4, 4), filters=("deflate",))
    p = str(tmp_path / "f.h5")
    w.save(p)
    raw = bytearray(open(p, "rb").read())
    # rewrite the deflate filter id (1) of the v1 pipeline message to an LZF-style third-party id
    i = raw.find(b"deflate\0")
    assert i > 0
    raw[i - 8:i - 6] = (32000).to_bytes(2, "little")
    open(p, "wb").write(bytes(raw))
    with pytest.raises(NotImplementedError, match="filter 32000"):
        slide_io.read_assets_from_h5(p)


def test_large_contiguous_read(tmp_path):
    """A 70k-tile slide's worth of features (70,000 x 1536 fp32 = 430 MB) reads in one copy."""
    if os.environ.get("GP_SKIP_LARGE_IO"):
        pytest.skip("GP_SKIP_LARGE_IO")
    n, dim = 70000, 1536
    feats = np.lib.stride_tricks.as_strided(np.arange(dim * 8, dtype=np.float32), (n, dim), (0, 4))
    feats = np.ascontiguousarray(feats) + np.arange(n, dtype=np.float32)[:, None]
    w = Writer()
    w.dataset("features", feats)
    w.dataset("coords", np.zeros((n, 2), np.int64))
    p = str(tmp_path / "big.h5")
    w.save(p)
    del w
    a, _ = slide_io.read_assets_from_h5(p)
    assert a["features"].shape == (n, dim)
    np.testing.assert_array_equal(a["features"][::9973], feats[::9973])


def test_against_h5py_when_available(tmp_path):
    h5py = pytest.importorskip("h5py")
    feats, coords = _slide(n=77)
    p = str(tmp_path / "h.h5")
    with h5py.File(p, "w") as f:
        f.create_dataset("features", data=feats, chunks=(16, 24), compression="gzip", shuffle=True)
        f.create_dataset("coords", data=coords)
        f["features"].attrs["patch_size"] = 256.0
        f["features"].attrs["name"] = "x"
    a, at = slide_io.read_assets_from_h5(p)
    np.testing.assert_array_equal(a["features"], feats)
    np.testing.assert_array_equal(a["coords"], coords)
    assert at["features"]["patch_size"] == 256.0 and at["features"]["name"] == "x"


def test_fletcher32_matches_spec_loop_and_known_answer():
    """The reader's vectorised Fletcher-32 equals the spec's block loop (h5_spec_writer) on edge
    lengths (odd, one 360-word block, several blocks, all-zero, all-0xff words) and the hand-computed
    value for b"abcdef" (big-endian words 0x6162 0x6364 0x6566: sum1 76332 mod 65535 = 0x2a2d,
    sum2 151636 mod 65535 = 0x5056); its 16-bit-half byte swap 0x56502d2a is the published
    little-endian-word Fletcher-32 of the same string."""
    from h5_spec_writer import fletcher32_spec
    assert slide_io.fletcher32(b"abcdef") == fletcher32_spec(b"abcdef") == 0x50562A2D
    rng = np.random.default_rng(9)
    for n in (0, 1, 2, 3, 719, 720, 721, 5000, 65537):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert slide_io.fletcher32(d) == fletcher32_spec(d), n
    for d in (b"\0" * 100, b"\xff" * 1000, b"\xff" * 1001):
        assert slide_io.fletcher32(d) == fletcher32_spec(d)


def test_fletcher32_corrupt_chunk_raises(tmp_path):
    feats = (np.arange(64 * 8, dtype=np.float32).reshape(64, 8) * 1.25 + 7.0)
    w = Writer("latest")
    w.dataset("features", feats, layout="chunked", chunks=(16, 8), filters=("fletcher32",))
    w.dataset("coords", np.zeros((64, 2), np.int64), layout="chunked", chunks=(16, 2), filters=("fletcher32",))
    p = str(tmp_path / "f.h5")
    w.save(p)
    assets, _ = slide_io.read_assets_from_h5(p)                 # intact file: checksums verify
    np.testing.assert_array_equal(assets["features"], feats)
    raw = bytearray(open(p, "rb").read())
    chunk = feats[16:32].tobytes()
    at = bytes(raw).find(chunk)
    assert at > 0
    raw[at + 37] ^= 0x10                                         # one flipped bit inside chunk 1
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ValueError, match="fletcher32 checksum mismatch"):
        slide_io.read_assets_from_h5(p)
