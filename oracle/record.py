"""CyberRT `.record` layout and the camera-topic extraction, restated in plain Python
-- test infrastructure only (tests/test_record.py builds synthetic records with it and
checks the C++ reader / writer, csrc/record.cpp, against it).

What it restates (parity unpinned: the reference's foreign/recordDeal.so is a prebuilt
Cython module whose source is absent and which wraps the third-party `cyber_record`
package [ext], not installed here; no .record fixture ships with the reference):
  * the published CyberRT file layout (apollo cyber/proto/record.proto,
    cyber/record/file/record_file_writer.cc): a 16-byte section header {int32 type,
    4 pad bytes, int64 size}; the Header section first, its message padded to 2048
    bytes (the writer's `blank` buffer: '0' then zeros); then Channel, ChunkHeader +
    ChunkBody pairs and finally the Index, whose SingleIndex entries hold each
    section's position and a cache (channel: message count, name, type; chunk header:
    message count, begin / end time, raw size; chunk body: message count); raw size
    is the running sum of the chunk's SingleMessage.content sizes, as Chunk::add
    (cyber/record/file/chunk) accumulates it, not the serialised body size;
  * protobuf wire encoding of those messages (field numbers from record.proto) and
    of apollo.drivers.CompressedImage (frame_id 2, format 3, data 4,
    measurement_time 5);
  * the extraction named by recordDeal's strings (combine_detect.py:839): per topic
    /drivers/camera/<camera>/compressed/image, the data of every message from the
    first key frame (an H.265 access unit with a VPS / SPS / PPS or IRAP NAL) on,
    concatenated into hevcs/<camera>.h265.
"""
import struct

HEADER, CHUNK_HEADER, CHUNK_BODY, INDEX, CHANNEL = 0, 1, 2, 3, 4
HEADER_LENGTH = 2048


# ---- protobuf wire format ----------------------------------------------------
def varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def field_varint(num, v):
    return varint(num << 3) + varint(v)


def field_bytes(num, b):
    return varint((num << 3) | 2) + varint(len(b)) + b


def field_double(num, x):
    return varint((num << 3) | 1) + struct.pack("<d", x)


def parse(b):
    """-> list of (num, wire type, value) in order (value: int or bytes)."""
    out, p = [], 0

    def rd():
        nonlocal p
        v, s = 0, 0
        while True:
            c = b[p]
            p += 1
            v |= (c & 0x7F) << s
            if not c & 0x80:
                return v
            s += 7
    while p < len(b):
        key = rd()
        num, wt = key >> 3, key & 7
        if wt == 0:
            out.append((num, wt, rd()))
        elif wt == 1:
            out.append((num, wt, struct.unpack_from("<Q", b, p)[0]))
            p += 8
        elif wt == 5:
            out.append((num, wt, struct.unpack_from("<I", b, p)[0]))
            p += 4
        elif wt == 2:
            n = rd()
            out.append((num, wt, bytes(b[p:p + n])))
            p += n
        else:
            raise ValueError("unsupported wire type")
    return out


def get(fields, num, default=None):
    for n, _, v in fields:
        if n == num:
            return v
    return default


# ---- messages ----------------------------------------------------------------
def compressed_image(data, frame_id="camera", fmt="h265", t=0.0):
    return field_bytes(2, frame_id.encode()) + field_bytes(3, fmt.encode()) + field_bytes(4, data) + field_double(5, t)


def single_message(channel, time_ns, content):
    return field_bytes(1, channel.encode()) + field_varint(2, time_ns) + field_bytes(3, content)


def section(kind, body):
    return struct.pack("<iiq", kind, 0, len(body)) + body


def write_record(channels, chunks, compress=0):
    """channels: [(name, message_type)]; chunks: [[(channel, time_ns, content bytes)]]
    -> bytes of a complete record, laid out as RecordFileWriter writes one: header,
    each channel before its first message, chunk header + body, index, header rewritten."""
    body = bytearray()
    pos = 16 + HEADER_LENGTH
    index, counts = [], {name: 0 for name, _ in channels}
    written = set()
    for ch in chunks:
        for name, mtype in channels:
            if name not in written and any(m[0] == name for m in ch):
                c = field_bytes(1, name.encode()) + field_bytes(2, mtype.encode()) + field_bytes(3, b"desc")
                index.append((CHANNEL, pos, name, mtype))
                body += section(CHANNEL, c)
                pos += 16 + len(c)
                written.add(name)
        cb = b"".join(field_bytes(1, single_message(*m)) for m in ch)
        t0, t1 = min(m[1] for m in ch), max(m[1] for m in ch)
        raw = sum(len(m[2]) for m in ch)          # Chunk::add: raw_size += message.content().size()
        chh = field_varint(1, t0) + field_varint(2, t1) + field_varint(3, len(ch)) + field_varint(4, raw)
        index.append((CHUNK_HEADER, pos, (len(ch), t0, t1, raw)))
        body += section(CHUNK_HEADER, chh)
        pos += 16 + len(chh)
        index.append((CHUNK_BODY, pos, len(ch)))
        body += section(CHUNK_BODY, cb)
        pos += 16 + len(cb)
        for m in ch:
            counts[m[0]] += 1
    entries = []
    for e in index:
        if e[0] == CHANNEL:
            cache = field_varint(1, counts[e[2]]) + field_bytes(2, e[2].encode()) + field_bytes(3, e[3].encode())
            entries.append(field_varint(1, e[0]) + field_varint(2, e[1]) + field_bytes(101, cache))
        elif e[0] == CHUNK_HEADER:
            n, t0, t1, raw = e[2]
            cache = field_varint(1, n) + field_varint(2, t0) + field_varint(3, t1) + field_varint(4, raw)
            entries.append(field_varint(1, e[0]) + field_varint(2, e[1]) + field_bytes(102, cache))
        else:
            entries.append(field_varint(1, e[0]) + field_varint(2, e[1]) + field_bytes(103, field_varint(1, e[2])))
    idx = b"".join(field_bytes(1, x) for x in entries)
    index_pos = pos
    body += section(INDEX, idx)
    size = pos + 16 + len(idx)
    times = [m[1] for ch in chunks for m in ch]
    hdr = (field_varint(1, 1) + field_varint(2, 0) + field_varint(3, compress) + field_varint(4, 20_000_000_000) +
           field_varint(5, 60_000_000_000) + field_varint(6, index_pos) + field_varint(7, len(chunks)) +
           field_varint(8, len(channels)) + field_varint(9, min(times)) + field_varint(10, max(times)) +
           field_varint(11, len(times)) + field_varint(12, size) + field_varint(13, 1) +
           field_varint(14, 200 * 1024 * 1024) + field_varint(15, 2048 * 1024 * 1024))
    pad = b"0" + bytes(HEADER_LENGTH - len(hdr) - 1)
    return section(HEADER, hdr) + pad + bytes(body)


def read_sections(data):
    """-> (header fields, [(type, position, body)])"""
    t, _, hs = struct.unpack_from("<iiq", data, 0)
    assert t == HEADER
    hdr = parse(data[16:16 + hs])
    secs, p = [], 16 + HEADER_LENGTH
    while p < len(data):
        t, _, n = struct.unpack_from("<iiq", data, p)
        secs.append((t, p, data[p + 16:p + 16 + n]))
        p += 16 + n
    return hdr, secs


def messages(data):
    """-> [(channel, time_ns, content bytes)] in file order"""
    out = []
    for t, _, b in read_sections(data)[1]:
        if t == CHUNK_BODY:
            for n, _, m in parse(b):
                f = parse(m)
                out.append((get(f, 1).decode(), get(f, 2), get(f, 3)))
    return out


# ---- H.265 access units ------------------------------------------------------
def nal_types(au):
    out, i = [], 0
    while True:
        i = au.find(b"\x00\x00\x01", i)
        if i < 0 or i + 4 >= len(au) + 1:
            return out
        if i + 3 < len(au):
            out.append((au[i + 3] >> 1) & 0x3F)
        i += 3


def is_key_frame(au):
    return any(16 <= t <= 23 or 32 <= t <= 34 for t in nal_types(au))


def camera_of(topic):
    return topic.split("/")[3]


def extract(record_blobs, topics):
    """-> {camera: bytes}: per topic, the data from its first key frame on."""
    out, started = {}, set()
    for data in record_blobs:
        for ch, _, content in messages(data):
            if ch not in topics:
                continue
            d = get(parse(content), 4)
            if ch not in started and not is_key_frame(d):
                continue
            started.add(ch)
            out[camera_of(ch)] = out.get(camera_of(ch), b"") + d
    return out
