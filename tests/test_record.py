"""`.record` container I/O (csrc/record.cpp through the C-ABI; vdmi.record mirrors
the reference's recordDeal.read_record2h265_all / write_allH265_record_all,
combine_detect.py:839, :958) against the Python restatement of the CyberRT layout
(oracle/record.py). No GPU.

Parity unpinned with the reference module itself: recordDeal.so is a prebuilt binary
(never run), cyber_record is absent and the reference ships no .record fixture; the
records here are synthetic, written by the oracle as CyberRT's RecordFileWriter lays
them out, with synthetic H.265 access units (Annex-B NAL units)."""
import os
import struct

import numpy as np
import pytest

from oracle import record as orec

CAMS = ["/drivers/camera/front_wide/compressed/image", "/drivers/camera/left_back/compressed/image",
        "/drivers/camera/rear/compressed/image"]
OTHER = "/apollo/sensor/gnss/best_pose"


def nal(t, payload):
    return b"\x00\x00\x00\x01" + bytes([t << 1, 1]) + payload


def au(rng, key, n=None):
    """one access unit: VPS/SPS/PPS + IDR slice (key) or a TRAIL_R slice, payload
    bytes 1..255 (no start-code emulation), first_slice_segment_in_pic_flag set"""
    n = int(rng.integers(20, 200)) if n is None else n
    body = bytes([0x80]) + bytes(rng.integers(1, 256, n, dtype=np.uint8))
    if key:
        return (nal(32, bytes(rng.integers(1, 256, 8, dtype=np.uint8))) + nal(33, bytes([1, 2, 3])) +
                nal(34, bytes([4, 5])) + nal(19, body))
    return nal(1, body)


def make_records(tmp, rng, segments=2, per_seg=12, lead=(2, 0, 3)):
    """segments of a record: each camera topic leads with `lead[i]` non-key units
    before its first key frame; a non-camera topic in between"""
    chans = [(c, "apollo.drivers.CompressedImage") for c in CAMS] + [(OTHER, "apollo.localization.Pose")]
    k = [0] * len(CAMS)
    blobs, names = [], []
    t = 1_000_000
    for s in range(segments):
        chunks = []
        for c in range(3):
            msgs = []
            for _ in range(per_seg // 3):
                for i, topic in enumerate(CAMS):
                    key = k[i] == lead[i] or (k[i] > lead[i] and (k[i] - lead[i]) % 5 == 0)
                    msgs.append((topic, t, orec.compressed_image(au(rng, key), frame_id=topic.split("/")[3])))
                    k[i] += 1
                    t += 1000
                msgs.append((OTHER, t, bytes(rng.integers(0, 256, 40, dtype=np.uint8))))
                t += 1000
            chunks.append(msgs)
        data = orec.write_record(chans, chunks)
        name = f"test.record.{s:05d}"
        with open(os.path.join(tmp, name), "wb") as f:
            f.write(data)
        blobs.append(data)
        names.append(name)
    return blobs, names


@pytest.fixture
def rec(tmp_path):
    rng = np.random.default_rng(3)
    src = tmp_path / "records"
    src.mkdir()
    blobs, names = make_records(str(src), rng)
    return tmp_path, src, blobs, names


def test_extract_matches_oracle(rec):
    from vdmi import record
    tmp, src, blobs, _ = rec
    n = record.read_record2h265_all(str(src), str(tmp / "h265"))
    exp = orec.extract(blobs, set(CAMS))
    assert n == len(exp) == 3
    for cam, data in exp.items():
        got = (tmp / "h265" / "hevcs" / f"{cam}.h265").read_bytes()
        assert got == data
        assert orec.is_key_frame(got[:300])            # starts at the first key frame


def test_repack_with_own_streams_is_byte_identical(rec):
    from vdmi import record
    tmp, src, blobs, names = rec
    record.read_record2h265_all(str(src), str(tmp / "h265"))
    vids = tmp / "videos"
    vids.mkdir()
    for f in (tmp / "h265" / "hevcs").iterdir():        # the extracted streams under the processed name
        (vids / (f.stem + "_processed.h265")).write_bytes(f.read_bytes())
    n = record.write_allH265_record_all(str(src), str(vids), str(tmp / "out"))
    assert n == len(names)
    for name, data in zip(names, blobs):
        assert (tmp / "out" / name).read_bytes() == data
        assert not (tmp / "out" / (name + ".tmp_record")).exists()


def test_repack_replaces_camera_data_and_relayouts(rec):
    """Desensitised streams with other access-unit sizes: exactly the extracted
    messages change (in order), every other message is untouched, and the layout
    (chunk raw sizes, index positions / caches, header size and index position)
    describes the new file."""
    from vdmi import record
    tmp, src, blobs, names = rec
    rng = np.random.default_rng(9)
    vids = tmp / "videos"
    vids.mkdir()
    orig = orec.extract(blobs, set(CAMS))
    new_aus = {}
    for cam in orig:
        # as many units as extracted messages, new payloads and lengths, same key pattern
        units = []
        for ch, _, content in [m for d in blobs for m in orec.messages(d)]:
            if ch.split("/")[3] != cam:
                continue
            units.append(orec.get(orec.parse(content), 4))
        first = next(i for i, u in enumerate(units) if orec.is_key_frame(u))
        repl = [au(rng, orec.is_key_frame(u), n=int(rng.integers(5, 400))) for u in units[first:]]
        new_aus[cam] = (first, repl)
        (vids / f"{cam}_processed.h265").write_bytes(b"".join(repl))
    record.write_allH265_record_all(str(src), str(vids), str(tmp / "out"))
    seen = {cam: 0 for cam in orig}
    for name, data in zip(names, blobs):
        out = (tmp / "out" / name).read_bytes()
        hdr, secs = orec.read_sections(out)
        assert orec.get(hdr, 12) == len(out)
        idx_sec = [s for s in secs if s[0] == orec.INDEX]
        assert len(idx_sec) == 1 and orec.get(hdr, 6) == idx_sec[0][1]
        by_pos = {p: (t, b) for t, p, b in secs}
        for e in orec.parse(idx_sec[0][2]):
            f = orec.parse(e[2])
            t, pos = orec.get(f, 1), orec.get(f, 2)
            assert by_pos[pos][0] == t
            if t == orec.CHUNK_HEADER:      # raw size = summed SingleMessage.content sizes (Chunk::add)
                raw = orec.get(orec.parse(orec.get(f, 102)), 4)
                nxt = [s for s in secs if s[1] > pos][0]
                content = sum(len(orec.get(orec.parse(m[2]), 3)) for m in orec.parse(nxt[2]))
                assert nxt[0] == orec.CHUNK_BODY and raw == content
                assert orec.get(orec.parse(by_pos[pos][1]), 4) == content
        a, b = orec.messages(data), orec.messages(out)
        assert [(c, t) for c, t, _ in a] == [(c, t) for c, t, _ in b]
        for (ch, _, ca), (_, _, cb) in zip(a, b):
            if ch not in CAMS:
                assert ca == cb
                continue
            cam = ch.split("/")[3]
            first, repl = new_aus[cam]
            k = seen[cam]
            seen[cam] += 1
            fa, fb = orec.parse(ca), orec.parse(cb)
            if k < first:
                assert ca == cb
            else:
                assert orec.get(fb, 4) == repl[k - first]
                assert [x for x in fa if x[0] != 4] == [x for x in fb if x[0] != 4]


def _new_streams(blobs, rng, vids, name="{cam}_processed.h265", cams=None):
    """one replacement access unit per extracted message, with new payloads / lengths"""
    orig = orec.extract(blobs, set(CAMS))
    out = {}
    for cam in orig:
        if cams is not None and cam not in cams:
            continue
        units = [orec.get(orec.parse(c), 4) for d in blobs for ch, _, c in orec.messages(d) if ch.split("/")[3] == cam]
        first = next(i for i, u in enumerate(units) if orec.is_key_frame(u))
        repl = [au(rng, orec.is_key_frame(u), n=int(rng.integers(5, 400))) for u in units[first:]]
        (vids / name.format(cam=cam)).write_bytes(b"".join(repl))
        out[cam] = (first, repl)
    return out


def test_repack_reference_output_names(rec):
    """combine_detect.py:658 names each desensitised stream <camera>_processed.<ext>
    in the directory it hands to write_allH265_record_all (:958): those are found and
    every extracted message is replaced."""
    from vdmi import record
    tmp, src, blobs, names = rec
    vids = tmp / "videos"
    vids.mkdir()
    new = _new_streams(blobs, np.random.default_rng(4), vids)
    assert record.write_allH265_record_all(str(src), str(vids), str(tmp / "out")) == len(names)
    for cam, (first, repl) in new.items():
        topic = f"/drivers/camera/{cam}/compressed/image"
        got = [orec.get(orec.parse(c), 4) for d in names for ch, _, c in orec.messages((tmp / "out" / d).read_bytes())
               if ch == topic]
        assert got[first:] == repl


def test_repack_from_extract_dir_is_an_error(rec):
    """The extract step writes the ORIGINAL streams as hevcs/<camera>.h265: a repack
    pointed at that directory must refuse (it would write the original frames back),
    and nothing is written."""
    import vdmi
    from vdmi import record
    tmp, src, blobs, names = rec
    record.read_record2h265_all(str(src), str(tmp / "h265"))
    with pytest.raises(vdmi.VdError, match="no desensitised stream"):
        record.write_allH265_record_all(str(src), str(tmp / "h265" / "hevcs"), str(tmp / "out"))
    assert not any((tmp / "out" / n).exists() for n in names)


def test_repack_short_stream_is_an_error(rec):
    """Fewer access units than extracted messages: refused, nothing written (a record
    with original frames left in would not be desensitised)."""
    import vdmi
    from vdmi import record
    tmp, src, blobs, names = rec
    vids = tmp / "videos"
    vids.mkdir()
    rng = np.random.default_rng(1)
    _new_streams(blobs, rng, vids)
    cam = CAMS[0].split("/")[3]
    (vids / f"{cam}_processed.h265").write_bytes(au(rng, True, n=50) + au(rng, False, n=60))
    with pytest.raises(vdmi.VdError, match="access units"):
        record.write_allH265_record_all(str(src), str(vids), str(tmp / "out"))
    assert not any((tmp / "out" / n).exists() for n in names)


def test_repack_missing_camera_stream_is_an_error(rec):
    import vdmi
    from vdmi import record
    tmp, src, blobs, names = rec
    vids = tmp / "videos"
    vids.mkdir()
    _new_streams(blobs, np.random.default_rng(2), vids, cams={CAMS[0].split("/")[3], CAMS[1].split("/")[3]})
    with pytest.raises(vdmi.VdError, match="no desensitised stream for camera rear"):
        record.write_allH265_record_all(str(src), str(vids), str(tmp / "out"))


def test_non_segment_files_are_skipped(rec):
    """Only <stem>.record and <stem>.record.<digits> are CyberRT segments."""
    from vdmi import record
    tmp, src, blobs, _ = rec
    (src / "notes.record.bak").write_bytes(b"junk" * 50)
    (src / "x.recording").write_bytes(b"junk" * 50)
    (src / "y.record.01a").write_bytes(b"junk" * 50)
    n = record.read_record2h265_all(str(src), str(tmp / "h265"))
    assert n == 3
    for cam, data in orec.extract(blobs, set(CAMS)).items():
        assert (tmp / "h265" / "hevcs" / f"{cam}.h265").read_bytes() == data


def test_record_errors(tmp_path):
    import vdmi
    from vdmi import record
    with pytest.raises(vdmi.VdError):
        record.read_record2h265_all(str(tmp_path / "missing"), str(tmp_path / "o"))
    d = tmp_path / "bad"
    d.mkdir()
    (d / "x.record").write_bytes(b"not a record" * 10)
    with pytest.raises(vdmi.VdError):
        record.read_record2h265_all(str(d), str(tmp_path / "o"))
    c = tmp_path / "comp"
    c.mkdir()
    chans = [(CAMS[0], "apollo.drivers.CompressedImage")]
    rng = np.random.default_rng(0)
    data = orec.write_record(chans, [[(CAMS[0], 1, orec.compressed_image(au(rng, True)))]], compress=2)
    (c / "y.record").write_bytes(data)
    with pytest.raises(vdmi.VdError, match="compressed"):
        record.read_record2h265_all(str(c), str(tmp_path / "o"))
    # a truncated section
    (c / "y.record").write_bytes(orec.write_record(chans, [[(CAMS[0], 1, orec.compressed_image(au(rng, True)))]])[:-7])
    with pytest.raises(vdmi.VdError):
        record.read_record2h265_all(str(c), str(tmp_path / "o"))


def test_oracle_layout_known_answer():
    """The section header and the header region as RecordFileWriter writes them:
    {int32 type, 4 zero bytes, int64 size}, the Header message, '0' then zeros to 2048."""
    data = orec.write_record([("/a", "T")], [[("/a", 5, b"xy")]])
    t, pad, n = struct.unpack_from("<iiq", data, 0)
    assert (t, pad) == (orec.HEADER, 0) and n < orec.HEADER_LENGTH
    assert data[16 + n:16 + n + 1] == b"0" and set(data[17 + n:16 + orec.HEADER_LENGTH]) == {0}
    hdr, secs = orec.read_sections(data)
    assert [s[0] for s in secs] == [orec.CHANNEL, orec.CHUNK_HEADER, orec.CHUNK_BODY, orec.INDEX]
    assert orec.get(hdr, 12) == len(data) and orec.get(hdr, 6) == secs[-1][1]
    assert orec.messages(data) == [("/a", 5, b"xy")]


def test_chunk_raw_size_is_summed_content_known_answer():
    """ChunkHeader.raw_size (and its index cache) = the sum of the chunk's
    SingleMessage.content sizes, as CyberRT's Chunk::add accumulates it."""
    data = orec.write_record([("/a", "T")], [[("/a", 5, b"xy"), ("/a", 6, b"abcde")]])
    hdr, secs = orec.read_sections(data)
    ch = orec.parse(secs[1][2])
    assert orec.get(ch, 4) == 7 and orec.get(ch, 3) == 2
    idx = [orec.parse(e[2]) for e in orec.parse(secs[-1][2])]
    cache = [orec.parse(orec.get(f, 102)) for f in idx if orec.get(f, 1) == orec.CHUNK_HEADER]
    assert orec.get(cache[0], 4) == 7
