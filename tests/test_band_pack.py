"""The packed band transfer format (csrc/band_pack.hip, include/sfrt.h "Band transfer
packing"): RGB + one alpha bit per pixel, lossless for frames whose alphas are 0 or 255
-- every frame of a world whose textures are (sfrt_world_alpha_binary; the reference's
Floor.png is, SphereWorld.cpp:376-381 keeps the texel's alpha).

CPU: the format restated in numpy below (the checker), the size function and the
argument checks that run before any launch.  GPU: sfrt_band_pack's bytes equal the
restatement's and sfrt_band_unpack inverts it, at ragged sizes; world alpha flags;
sfrt_multi frames are the same bytes packed or not (tests/test_gpu_bands.py covers the
golden frames with the default, packing, transfer)."""
import ctypes

import numpy as np
import pytest

import scenes

BLOCK = 256


@pytest.fixture(scope="module")
def lib(built):
    import sfrt
    return sfrt.lib()


def pack_reference(px: np.ndarray) -> np.ndarray:
    """uint32 RGBA pixels (R in the low byte) -> packed bytes: per the header, B = ceil(P /
    256) blocks, RGB of pixel p at 3p, then the little-endian bit string of alpha == 255."""
    p = px.size
    b = -(-p // BLOCK)
    rgb = np.zeros(b * BLOCK * 3, np.uint8)
    by = px.view(np.uint8).reshape(-1, 4)
    rgb[:3 * p] = by[:, :3].ravel()
    bits = np.zeros(b * BLOCK, np.uint8)
    bits[:p] = by[:, 3] == 255
    return np.concatenate([rgb, np.packbits(bits, bitorder="little")])


def unpack_reference(packed: np.ndarray, p: int) -> np.ndarray:
    b = -(-p // BLOCK)
    rgb = packed[:b * BLOCK * 3][:3 * p].reshape(-1, 3)
    bits = np.unpackbits(packed[b * BLOCK * 3:], bitorder="little")[:p]
    out = np.empty((p, 4), np.uint8)
    out[:, :3] = rgb
    out[:, 3] = np.where(bits == 1, 255, 0)
    return out.ravel().view(np.uint32)


def _pixels(p, seed, alphas=(0, 255)):
    rng = np.random.default_rng(seed)
    by = rng.integers(0, 256, size=(p, 4), dtype=np.uint8)
    by[:, 3] = rng.choice(np.array(alphas, np.uint8), size=p)
    return by.ravel().view(np.uint32)


SIZES = [1, 3, 4, 5, 63, 64, 255, 256, 257, 1000, 3840 * 8 + 5, (1 << 20) + 3]


@pytest.mark.parametrize("p", SIZES)
def test_reference_format_round_trip(p):
    px = _pixels(p, p)
    packed = pack_reference(px)
    assert packed.size == -(-p // BLOCK) * 800
    assert np.array_equal(unpack_reference(packed, p), px)


def test_packed_bytes_and_argument_checks(lib):
    """Host-only paths: sizes, and invalid arguments refused before any launch."""
    f = lib.sfrt_band_packed_bytes
    for p in [0] + SIZES + [16384 * 16384]:
        assert f(p) == -(-p // BLOCK) * 800, p
    assert f(-1) < 0
    vp = ctypes.c_void_p
    pack = lambda rgba, p, packed: lib.sfrt_band_pack(rgba, p, packed, None)  # noqa: E731
    unpack = lambda rgba, p, packed: lib.sfrt_band_unpack(packed, p, rgba, None)  # noqa: E731
    for fn in (pack, unpack):
        assert fn(None, 0, None) == 0                          # nothing to do
        assert fn(None, -1, None) == -1                        # negative size
        assert fn(None, 4, vp(0x1000)) == -1                   # null RGBA buffer
        assert fn(vp(0x1000), 4, None) == -1                   # null packed buffer
        assert fn(vp(0x1002), 4, vp(0x2000)) == -1             # RGBA not 4-byte aligned
        assert fn(vp(0x1000), 4, vp(0x2004)) == -1             # packed not 8-byte aligned


@pytest.mark.gpu
@pytest.mark.parametrize("p", SIZES + [3840 * 2160])
def test_gpu_pack_matches_format_and_inverts(built, p):
    import torch

    import sfrt
    px = _pixels(p, 7 * p + 1)
    src = torch.from_numpy(px.view(np.int32).copy()).cuda()
    nbytes = sfrt.band_packed_bytes(p)
    packed = torch.full((nbytes,), 0x5A, dtype=torch.uint8, device="cuda")
    back = torch.full((p,), 0x11223344, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    sfrt.band_pack(src.data_ptr(), p, packed.data_ptr(), s)
    sfrt.band_unpack(packed.data_ptr(), p, back.data_ptr(), s)
    torch.cuda.synchronize()
    assert np.array_equal(packed.cpu().numpy(), pack_reference(px))
    assert np.array_equal(back.cpu().numpy().view(np.uint32), px)


@pytest.mark.gpu
def test_gpu_unpack_leaves_pixels_past_the_band(built):
    """Unpacking P pixels writes exactly P dwords (the frame rows after a band survive)."""
    import torch

    import sfrt
    p = 1001
    px = _pixels(p, 3)
    src = torch.from_numpy(px.view(np.int32).copy()).cuda()
    packed = torch.empty(sfrt.band_packed_bytes(p), dtype=torch.uint8, device="cuda")
    out = torch.full((p + 64,), -1, dtype=torch.int32, device="cuda")
    sfrt.band_pack(src.data_ptr(), p, packed.data_ptr())
    sfrt.band_unpack(packed.data_ptr(), p, out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got[:p], px)
    assert (got[p:] == 0xFFFFFFFF).all()


@pytest.mark.gpu
def test_world_alpha_binary(built):
    """The reference's Floor.png is alpha-binary; a texture with a translucent texel is not;
    a world without textures is not."""
    import sfrt
    rgba, tw, th = scenes.load_floor()
    a = np.asarray(rgba, np.uint8).reshape(-1, 4)
    assert set(np.unique(a[:, 3])) <= {0, 255}
    with sfrt.World(0) as w:
        assert not w.alpha_binary()
        w.load_texture(rgba, tw, th)
        assert w.alpha_binary()
        odd = a.copy()
        odd[5, 3] = 128
        w.load_texture(odd.ravel(), tw, th, slot=2)
        assert not w.alpha_binary()
        w.load_texture(rgba, tw, th, slot=2)
        assert w.alpha_binary()


@pytest.mark.gpu
def test_rendered_frames_pack_losslessly(built):
    """A 4K lcg64 frame and a 1080p default10 frame survive pack + unpack byte for byte."""
    import torch

    import sfrt
    floor = scenes.load_floor()
    for sc, wd, ht in ((scenes.lcg64(), 3840, 2160), (scenes.default10().posed(0.7, 0.3), 1920, 1080)):
        with sfrt.World(0) as w:
            w.load_texture(*floor)
            w.set_scene(sc, wd, ht)
            frame = torch.empty(ht, wd * 4, dtype=torch.uint8, device="cuda")
            w.render_band(frame.data_ptr(), wd * 4, 0, ht)
            w.check()
            packed = torch.empty(sfrt.band_packed_bytes(wd * ht), dtype=torch.uint8, device="cuda")
            back = torch.empty_like(frame)
            sfrt.band_pack(frame.data_ptr(), wd * ht, packed.data_ptr())
            sfrt.band_unpack(packed.data_ptr(), wd * ht, back.data_ptr())
            torch.cuda.synchronize()
            assert torch.equal(frame, back)


@pytest.mark.gpu
@pytest.mark.parametrize("transport,width", [(1, 1000), (2, 1000), (2, 1001)])
def test_multi_transfer_formats_same_frame(built, transport, width):
    """sfrt_multi: RGBA and packed transfers give the same frame, equal and unequal bands
    (a 1001-pixel row makes band sizes that are not whole 4-pixel groups); AUTO packs an
    alpha-binary world and not one with a translucent texel; PACKED refuses it."""
    import sfrt
    rgba, tw, th = scenes.load_floor()
    height = 563
    devs = [0] if transport == sfrt.SFRT_MULTI_RCCL else [0, 0, 0]
    sc = scenes.lcg64().posed(0.4, 0.1)
    with sfrt.World(0) as ref:
        ref.load_texture(rgba, tw, th)
        ref.set_scene(sc, width, height)
        want = ref.render()
    with sfrt.Multi(devs, transport) as m:
        m.load_texture(rgba, tw, th)
        m.set_scene(sc, width, height)
        for rows in (None, [r for _, r in sfrt.multi_bands(height, len(devs), 2.0)]):
            m.set_bands(rows)
            for fmt in (sfrt.SFRT_TRANSFER_RGBA, sfrt.SFRT_TRANSFER_PACKED, sfrt.SFRT_TRANSFER_AUTO):
                m.set_transfer(fmt)
                assert np.array_equal(m.update_image(), want), (rows, fmt)
                assert m.transfer() == (fmt, fmt != sfrt.SFRT_TRANSFER_RGBA and len(devs) > 1)
        odd = np.asarray(rgba, np.uint8).reshape(-1, 4).copy()
        odd[0, 3] = 77
        m.load_texture(odd.ravel(), tw, th, slot=1)
        m.set_transfer(sfrt.SFRT_TRANSFER_AUTO)
        assert np.array_equal(m.update_image(), want)
        assert m.transfer() == (sfrt.SFRT_TRANSFER_AUTO, False)
        if len(devs) > 1:
            m.set_transfer(sfrt.SFRT_TRANSFER_PACKED)
            with pytest.raises(sfrt.SfrtError):
                m.update_image()
