// record.cpp — Apollo CyberRT .record container I/O for the camera topics, on the host.
//
// Replaces the reference's prebuilt Cython module foreign/recordDeal.so (called at
// /root/reference/combine_detect.py:839 `recordDeal.read_record2h265_all(record_dir,
// output_h265_dir)` and :958 `recordDeal.write_allH265_record_all(record_dir,
// output_videos_dir, record_output_dir)`; the module wraps the third-party
// `cyber_record` reader, absent here). The module's strings name the twelve
// `/drivers/camera/<camera>/compressed/image` topics, an `<out>/hevcs` directory of
// `.h265` files, key-frame handling and an intermediate `.tmp_record`; its source is
// not in the reference, so the behaviour below is restated from those names and from
// the published CyberRT record layout (cyber/proto/record.proto, cyber/record/file):
//
//   file    = Section{HEADER} Header [padding to 2048 B] then sections to EOF:
//             Section{CHANNEL} Channel | Section{CHUNK_HEADER} ChunkHeader |
//             Section{CHUNK_BODY} ChunkBody | Section{INDEX} Index
//   Section = int32 type, 4 zero bytes, int64 size (16 B, little-endian)
//   ChunkBody.messages (1) = SingleMessage{channel_name 1, time 2, content 3}
//   content of a camera topic = apollo.drivers.CompressedImage, H.265 access unit in
//   field 4 (data)
//
// extract: for each camera topic, in file order over the record's segments, the data
//   of every message from the topic's first key frame (an access unit holding a VPS /
//   SPS / PPS or IRAP slice NAL) on, concatenated into <out>/hevcs/<camera>.h265.
// repack:  the same records rewritten with each extracted message's data replaced by
//   the matching access unit of <videos>/<camera>_processed.h265 (the name the
//   reference's create_video gives it, combine_detect.py:658; <camera>.h265 also
//   accepted), the desensitised stream split at access-unit boundaries; a topic with
//   extracted messages and no stream, or a stream whose access-unit count differs
//   from the topic's extracted message count, is an error (no record is written with
//   original frames left in). Every other byte is carried over, and the positions /
//   sizes that move (chunk raw sizes = summed message content sizes, index positions
//   and caches, header size and index position) are recomputed. Written as
//   <name>.tmp_record, then renamed.
// Protobuf messages are edited as field lists and re-serialised in their original
// field order, so a record written by a canonical protobuf encoder and repacked with
// its own extracted streams comes back byte-identical (tests/test_record.py).
// Compressed records (Header.compress = BZ2 / LZ4) are rejected: no codec library here.
#include "../../include/vdmi.h"
#include "vd_common.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <map>
#include <string>
#include <sys/stat.h>
#include <vector>

namespace {

enum { SEC_HEADER = 0, SEC_CHUNK_HEADER = 1, SEC_CHUNK_BODY = 2, SEC_INDEX = 3, SEC_CHANNEL = 4 };
constexpr size_t kHeaderLength = 2048;

const char* const kTopics[] = {
    "/drivers/camera/front_narrow/compressed/image", "/drivers/camera/front_wide/compressed/image",
    "/drivers/camera/front_wide_left/compressed/image", "/drivers/camera/left_front/compressed/image",
    "/drivers/camera/left_back/compressed/image", "/drivers/camera/right_front/compressed/image",
    "/drivers/camera/right_back/compressed/image", "/drivers/camera/rear/compressed/image",
    "/drivers/camera/surround_front/compressed/image", "/drivers/camera/surround_rear/compressed/image",
    "/drivers/camera/surround_left/compressed/image", "/drivers/camera/surround_right/compressed/image",
};
constexpr int kNumTopics = sizeof(kTopics) / sizeof(kTopics[0]);

int topic_index(const std::string& ch) {
    for (int i = 0; i < kNumTopics; ++i)
        if (ch == kTopics[i]) return i;
    return -1;
}

std::string camera_of(int t) {   // "/drivers/camera/<camera>/compressed/image" -> <camera>
    const std::string s = kTopics[t];
    const size_t a = std::strlen("/drivers/camera/"), b = s.find('/', a);
    return s.substr(a, b - a);
}

// ---- protobuf wire format: a message as an ordered list of fields ----------------
struct Field {
    uint32_t num;
    uint32_t wt;           // 0 varint, 1 fixed64, 2 length-delimited, 5 fixed32
    uint64_t v;            // wt 0 / 1 / 5
    std::string b;         // wt 2
};

bool get_varint(const uint8_t*& p, const uint8_t* e, uint64_t& v) {
    v = 0;
    for (int s = 0; s < 64; s += 7) {
        if (p >= e) return false;
        const uint8_t c = *p++;
        v |= (uint64_t)(c & 0x7F) << s;
        if (!(c & 0x80)) return true;
    }
    return false;
}

void put_varint(std::string& o, uint64_t v) {
    while (v >= 0x80) { o.push_back((char)((v & 0x7F) | 0x80)); v >>= 7; }
    o.push_back((char)v);
}

bool parse(const std::string& s, std::vector<Field>& out) {
    const uint8_t* p = (const uint8_t*)s.data();
    const uint8_t* e = p + s.size();
    out.clear();
    while (p < e) {
        uint64_t key;
        if (!get_varint(p, e, key)) return false;
        Field f{(uint32_t)(key >> 3), (uint32_t)(key & 7), 0, {}};
        if (f.num == 0) return false;
        if (f.wt == 0) {
            if (!get_varint(p, e, f.v)) return false;
        } else if (f.wt == 1 || f.wt == 5) {
            const int n = f.wt == 1 ? 8 : 4;
            if (e - p < n) return false;
            std::memcpy(&f.v, p, n);
            p += n;
        } else if (f.wt == 2) {
            uint64_t n;
            if (!get_varint(p, e, n) || (uint64_t)(e - p) < n) return false;
            f.b.assign((const char*)p, (size_t)n);
            p += n;
        } else {
            return false;                                  // groups: not in these messages
        }
        out.push_back(std::move(f));
    }
    return true;
}

std::string serialize(const std::vector<Field>& fs) {
    std::string o;
    for (const Field& f : fs) {
        put_varint(o, ((uint64_t)f.num << 3) | f.wt);
        if (f.wt == 0) put_varint(o, f.v);
        else if (f.wt == 1) o.append((const char*)&f.v, 8);
        else if (f.wt == 5) o.append((const char*)&f.v, 4);
        else { put_varint(o, f.b.size()); o += f.b; }
    }
    return o;
}

Field* find(std::vector<Field>& fs, uint32_t num) {
    for (Field& f : fs)
        if (f.num == num) return &f;
    return nullptr;
}

// ---- record file -----------------------------------------------------------------
struct Section {
    int32_t type;
    uint64_t pos;          // byte offset of the section header in the file
    std::string body;
};

struct Record {
    std::string header;    // Header message
    std::string pad;       // the header region's bytes after the message
    std::vector<Section> secs;
};

int read_file(const std::string& path, std::string& data) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return vd_set_error(VD_ERR_ARG, "record: cannot open %s", path.c_str());
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    data.resize(n > 0 ? (size_t)n : 0);
    const size_t got = n > 0 ? std::fread(&data[0], 1, (size_t)n, f) : 0;
    std::fclose(f);
    if (got != data.size()) return vd_set_error(VD_ERR_ARG, "record: short read of %s", path.c_str());
    return VD_OK;
}

bool sec_at(const std::string& d, size_t at, int32_t& type, uint64_t& size) {
    if (d.size() < at + 16) return false;
    std::memcpy(&type, d.data() + at, 4);
    int64_t s;
    std::memcpy(&s, d.data() + at + 8, 8);
    if (s < 0 || (uint64_t)s > d.size() - at - 16) return false;
    size = (uint64_t)s;
    return true;
}

int load_record(const std::string& path, Record& r) {
    std::string d;
    int rc = read_file(path, d);
    if (rc) return rc;
    int32_t t;
    uint64_t hs;
    if (!sec_at(d, 0, t, hs) || t != SEC_HEADER || hs > kHeaderLength || d.size() < 16 + kHeaderLength)
        return vd_set_error(VD_ERR_ARG, "record: %s has no CyberRT header section", path.c_str());
    r.header.assign(d, 16, (size_t)hs);
    r.pad.assign(d, 16 + (size_t)hs, kHeaderLength - (size_t)hs);
    std::vector<Field> hf;
    if (!parse(r.header, hf)) return vd_set_error(VD_ERR_ARG, "record: %s: bad header message", path.c_str());
    if (const Field* c = find(hf, 3))
        if (c->v != 0) return vd_set_error(VD_ERR_ARG, "record: %s is compressed (type %d), not supported", path.c_str(), (int)c->v);
    size_t at = 16 + kHeaderLength;
    r.secs.clear();
    while (at < d.size()) {
        uint64_t sz;
        if (!sec_at(d, at, t, sz)) return vd_set_error(VD_ERR_ARG, "record: %s: truncated section at %zu", path.c_str(), at);
        if (t < SEC_CHUNK_HEADER || t > SEC_CHANNEL)
            return vd_set_error(VD_ERR_ARG, "record: %s: unknown section type %d at %zu", path.c_str(), t, at);
        r.secs.push_back(Section{t, at, d.substr(at + 16, (size_t)sz)});
        at += 16 + (size_t)sz;
    }
    return VD_OK;
}

void put_section(std::string& o, int32_t type, size_t size) {
    char h[16] = {0};
    std::memcpy(h, &type, 4);
    const int64_t s = (int64_t)size;
    std::memcpy(h + 8, &s, 8);
    o.append(h, 16);
}

// H.265 Annex-B: NAL unit types of every NAL in a buffer, with their byte ranges
struct Nal { size_t start, end; int type; bool first_slice; };

std::vector<Nal> nals(const std::string& s) {
    std::vector<Nal> out;
    const uint8_t* p = (const uint8_t*)s.data();
    const size_t n = s.size();
    std::vector<size_t> sc;                               // start-code positions (first zero byte)
    for (size_t i = 0; i + 3 <= n; ++i) {
        if (p[i] == 0 && p[i + 1] == 0 && p[i + 2] == 1) {
            sc.push_back(i > 0 && p[i - 1] == 0 ? i - 1 : i);
            i += 2;
        }
    }
    for (size_t k = 0; k < sc.size(); ++k) {
        size_t h = sc[k];
        while (p[h] == 0) ++h;                            // skip 00 00 (00) to 01
        ++h;                                              // NAL header
        const size_t end = k + 1 < sc.size() ? sc[k + 1] : n;
        if (h + 2 > end) continue;
        const int type = (p[h] >> 1) & 0x3F;
        const bool fs = type < 32 && h + 2 < end && (p[h + 2] & 0x80);
        out.push_back(Nal{sc[k], end, type, fs});
    }
    return out;
}

bool is_key_frame(const std::string& au) {
    for (const Nal& x : nals(au))
        if ((x.type >= 16 && x.type <= 23) || (x.type >= 32 && x.type <= 34)) return true;   // IRAP / VPS / SPS / PPS
    return false;
}

// access units of an elementary stream: a new unit starts at an AUD / VPS / SPS / PPS /
// prefix SEI or at a slice with first_slice_segment_in_pic_flag, once the current unit
// holds a slice
std::vector<std::string> access_units(const std::string& s) {
    std::vector<std::string> out;
    const std::vector<Nal> ns = nals(s);
    size_t au0 = 0;
    bool have_vcl = false;
    for (const Nal& x : ns) {
        const bool vcl = x.type < 32;
        const bool starts = x.type == 35 || (x.type >= 32 && x.type <= 34) || x.type == 39 || (vcl && x.first_slice);
        if (starts && have_vcl) {
            out.push_back(s.substr(au0, x.start - au0));
            au0 = x.start;
            have_vcl = false;
        }
        if (vcl) have_vcl = true;
    }
    if (have_vcl || au0 < s.size()) out.push_back(s.substr(au0));
    return out;
}

// CyberRT segment names: <stem>.record or <stem>.record.<digits> (the recorder's
// split segments); anything else (foo.record.bak, x.recording, .tmp_record) is skipped
bool is_segment_name(const std::string& name) {
    const size_t k = name.rfind(".record");
    if (k == std::string::npos || k == 0) return false;
    const size_t e = k + 7;
    if (e == name.size()) return true;
    if (name[e] != '.' || e + 1 == name.size()) return false;
    for (size_t i = e + 1; i < name.size(); ++i)
        if (name[i] < '0' || name[i] > '9') return false;
    return true;
}

int list_records(const char* dir, std::vector<std::string>& files) {
    DIR* d = opendir(dir);
    if (!d) return vd_set_error(VD_ERR_ARG, "record: cannot open directory %s", dir);
    while (dirent* e = readdir(d)) {
        const std::string name = e->d_name;
        if (!is_segment_name(name)) continue;
        const std::string path = std::string(dir) + "/" + name;
        struct stat st;
        if (stat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode)) files.push_back(name);
    }
    closedir(d);
    std::sort(files.begin(), files.end());
    if (files.empty()) return vd_set_error(VD_ERR_ARG, "record: no .record files in %s", dir);
    return VD_OK;
}

int write_file(const std::string& path, const std::string& data) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return vd_set_error(VD_ERR_ARG, "record: cannot write %s", path.c_str());
    const size_t put = std::fwrite(data.data(), 1, data.size(), f);
    const bool ok = put == data.size() && std::fclose(f) == 0;
    if (!ok) return vd_set_error(VD_ERR_ARG, "record: write of %s failed", path.c_str());
    return VD_OK;
}

void make_dirs(const std::string& p) {
    for (size_t i = 1; i <= p.size(); ++i)
        if (i == p.size() || p[i] == '/') mkdir(p.substr(0, i).c_str(), 0755);
}

// calls fn(topic, message fields, content fields) for every camera-topic message in
// file order; fn may edit the content fields (returns true if it did)
template <class Fn>
int for_camera_messages(Record& r, Fn&& fn, bool rewrite) {
    for (Section& s : r.secs) {
        if (s.type != SEC_CHUNK_BODY) continue;
        std::vector<Field> body;
        if (!parse(s.body, body)) return vd_set_error(VD_ERR_ARG, "record: bad chunk body at %llu", (unsigned long long)s.pos);
        bool changed = false;
        for (Field& m : body) {
            if (m.num != 1 || m.wt != 2) continue;
            std::vector<Field> msg;
            if (!parse(m.b, msg)) return vd_set_error(VD_ERR_ARG, "record: bad message at %llu", (unsigned long long)s.pos);
            const Field* ch = find(msg, 1);
            if (!ch || ch->wt != 2) continue;
            const int t = topic_index(ch->b);
            if (t < 0) continue;
            Field* content = find(msg, 3);
            if (!content || content->wt != 2) continue;
            std::vector<Field> img;
            if (!parse(content->b, img)) continue;        // not a CompressedImage: left alone
            if (fn(t, img) && rewrite) {
                content->b = serialize(img);
                m.b = serialize(msg);
                changed = true;
            }
        }
        if (changed) s.body = serialize(body);
    }
    return VD_OK;
}

// ChunkHeader.raw_size as CyberRT's Chunk::add keeps it: the running sum of the
// chunk's SingleMessage.content sizes (not the serialised body size)
int content_bytes(const std::string& body, uint64_t& total) {
    std::vector<Field> fs;
    if (!parse(body, fs)) return vd_set_error(VD_ERR_ARG, "record: bad chunk body");
    total = 0;
    for (Field& m : fs) {
        if (m.num != 1 || m.wt != 2) continue;
        std::vector<Field> msg;
        if (!parse(m.b, msg)) return vd_set_error(VD_ERR_ARG, "record: bad message in chunk body");
        if (const Field* c = find(msg, 3))
            if (c->wt == 2) total += c->b.size();
    }
    return VD_OK;
}

// positions and sizes after bodies changed: chunk headers' raw_size, the index's
// positions and chunk-header caches, the header's size and index position
int relayout(Record& r, std::string& out) {
    std::map<uint64_t, uint64_t> moved;                   // old section position -> new
    std::map<uint64_t, uint64_t> body_size;               // old position of a chunk header -> its raw size
    uint64_t at = 16 + kHeaderLength;
    for (size_t i = 0; i < r.secs.size(); ++i) {
        Section& s = r.secs[i];
        if (s.type == SEC_CHUNK_HEADER && i + 1 < r.secs.size() && r.secs[i + 1].type == SEC_CHUNK_BODY) {
            uint64_t raw_size = 0;
            int rc = content_bytes(r.secs[i + 1].body, raw_size);
            if (rc) return rc;
            body_size[s.pos] = raw_size;
            std::vector<Field> ch;
            if (parse(s.body, ch)) {
                if (Field* raw = find(ch, 4)) {
                    raw->v = raw_size;
                    s.body = serialize(ch);
                }
            }
        }
        moved[s.pos] = at;
        at += 16 + s.body.size();
    }
    uint64_t index_pos = 0;
    for (Section& s : r.secs) {
        if (s.type != SEC_INDEX) continue;
        index_pos = moved[s.pos];
        std::vector<Field> idx;
        if (!parse(s.body, idx)) return vd_set_error(VD_ERR_ARG, "record: bad index section");
        for (Field& e : idx) {
            if (e.num != 1 || e.wt != 2) continue;
            std::vector<Field> si;
            if (!parse(e.b, si)) return vd_set_error(VD_ERR_ARG, "record: bad index entry");
            Field* pos = find(si, 2);
            if (!pos) continue;
            const uint64_t old = pos->v;
            const auto it = moved.find(old);
            if (it != moved.end()) pos->v = it->second;
            if (Field* cache = find(si, 102)) {            // ChunkHeaderCache.raw_size
                std::vector<Field> c;
                const auto bs = body_size.find(old);
                if (bs != body_size.end() && parse(cache->b, c)) {
                    if (Field* raw = find(c, 4)) raw->v = bs->second;
                    cache->b = serialize(c);
                }
            }
            e.b = serialize(si);
        }
        s.body = serialize(idx);
    }
    // re-serialising the index may change its size (varint widths); it is the last
    // section of a complete record, so only the file size and its own position follow
    at = 16 + kHeaderLength;
    for (Section& s : r.secs) {
        if (s.type == SEC_INDEX) index_pos = at;
        at += 16 + s.body.size();
    }
    std::vector<Field> hf;
    if (!parse(r.header, hf)) return vd_set_error(VD_ERR_ARG, "record: bad header message");
    if (Field* f = find(hf, 6)) f->v = index_pos;
    if (Field* f = find(hf, 12)) f->v = at;
    const std::string h = serialize(hf);
    if (h.size() > kHeaderLength) return vd_set_error(VD_ERR_ARG, "record: header larger than %zu B", kHeaderLength);
    out.clear();
    out.reserve((size_t)at);
    put_section(out, SEC_HEADER, h.size());
    out += h;
    std::string pad = r.pad;
    pad.resize(kHeaderLength - h.size(), '\0');
    out += pad;
    for (const Section& s : r.secs) {
        put_section(out, s.type, s.body.size());
        out += s.body;
    }
    return VD_OK;
}

}  // namespace

extern "C" int vd_record_extract_h265(const char* record_dir, const char* out_dir, int* topics_written) {
    if (!record_dir || !out_dir) return vd_set_error(VD_ERR_ARG, "vd_record_extract_h265: null path");
    std::vector<std::string> files;
    int rc = list_records(record_dir, files);
    if (rc) return rc;
    std::vector<std::string> stream(kNumTopics);
    std::vector<int> started(kNumTopics, 0), seen(kNumTopics, 0);
    for (const std::string& name : files) {
        Record r;
        if ((rc = load_record(std::string(record_dir) + "/" + name, r))) return rc;
        rc = for_camera_messages(r, [&](int t, std::vector<Field>& img) {
            seen[t] = 1;
            const Field* data = find(img, 4);
            if (!data || data->wt != 2) return false;
            if (!started[t] && !is_key_frame(data->b)) return false;   // the stream starts at a key frame
            started[t] = 1;
            stream[t] += data->b;
            return false;
        }, false);
        if (rc) return rc;
    }
    const std::string hdir = std::string(out_dir) + "/hevcs";
    make_dirs(hdir);
    int n = 0;
    for (int t = 0; t < kNumTopics; ++t) {
        if (!started[t]) continue;
        if ((rc = write_file(hdir + "/" + camera_of(t) + ".h265", stream[t]))) return rc;
        ++n;
    }
    if (topics_written) *topics_written = n;
    return VD_OK;
}

extern "C" int vd_record_repack_h265(const char* record_dir, const char* videos_dir, const char* out_dir,
                                     int* records_written) {
    if (!record_dir || !videos_dir || !out_dir) return vd_set_error(VD_ERR_ARG, "vd_record_repack_h265: null path");
    std::vector<std::string> files;
    int rc = list_records(record_dir, files);
    if (rc) return rc;
    // per camera topic, how many messages the extract step put into its stream
    std::vector<size_t> count(kNumTopics, 0);
    {
        std::vector<int> started(kNumTopics, 0);
        for (const std::string& name : files) {
            Record r;
            if ((rc = load_record(std::string(record_dir) + "/" + name, r))) return rc;
            rc = for_camera_messages(r, [&](int t, std::vector<Field>& img) {
                const Field* data = find(img, 4);
                if (!data || data->wt != 2) return false;
                if (!started[t] && !is_key_frame(data->b)) return false;
                started[t] = 1;
                ++count[t];
                return false;
            }, false);
            if (rc) return rc;
        }
    }
    // the desensitised streams (combine_detect.py:658 writes <camera>_processed.<ext>),
    // split into access units; every extracted topic needs one with exactly one access
    // unit per extracted message -- a record is never written with original frames left in
    std::vector<std::vector<std::string>> aus(kNumTopics);
    std::vector<int> have(kNumTopics, 0);
    for (int t = 0; t < kNumTopics; ++t) {
        if (!count[t]) continue;
        // only the desensitised names: <camera>.h265 is what vd_record_extract_h265 writes
        // for the ORIGINAL stream (hevcs/<camera>.h265), so accepting it would let a repack
        // pointed at the extract directory put the original frames back
        for (const char* pat : {"%s/%s_processed.h265", "%s/%s_processed.hevc", "%s/processed_%s.h265"}) {
            char p[4096];
            std::snprintf(p, sizeof p, pat, videos_dir, camera_of(t).c_str());
            struct stat st;
            if (stat(p, &st) != 0) continue;
            std::string s;
            if ((rc = read_file(p, s))) return rc;
            aus[t] = access_units(s);
            have[t] = 1;
            if (aus[t].size() != count[t])
                return vd_set_error(VD_ERR_ARG, "record: %s holds %zu access units but the records hold %zu extracted "
                                    "messages of camera %s", p, aus[t].size(), count[t], camera_of(t).c_str());
            break;
        }
        if (!have[t])
            return vd_set_error(VD_ERR_ARG, "record: no desensitised stream for camera %s in %s (looked for "
                                "%s_processed.h265 / .hevc, processed_%s.h265; the un-suffixed %s.h265 is the extracted "
                                "original and is never used)", camera_of(t).c_str(), videos_dir,
                                camera_of(t).c_str(), camera_of(t).c_str(), camera_of(t).c_str());
    }
    make_dirs(out_dir);
    std::vector<size_t> next(kNumTopics, 0);
    std::vector<int> started(kNumTopics, 0);
    int n = 0;
    for (const std::string& name : files) {
        Record r;
        if ((rc = load_record(std::string(record_dir) + "/" + name, r))) return rc;
        rc = for_camera_messages(r, [&](int t, std::vector<Field>& img) {
            if (!have[t]) return false;
            Field* data = find(img, 4);
            if (!data || data->wt != 2) return false;
            if (!started[t] && !is_key_frame(data->b)) return false;   // not in the extracted stream
            started[t] = 1;
            data->b = aus[t][next[t]++];                            // counts checked above
            return true;
        }, true);
        if (rc) return rc;
        std::string out;
        if ((rc = relayout(r, out))) return rc;
        const std::string tmp = std::string(out_dir) + "/" + name + ".tmp_record";
        if ((rc = write_file(tmp, out))) return rc;
        const std::string dst = std::string(out_dir) + "/" + name;
        if (std::rename(tmp.c_str(), dst.c_str()) != 0) return vd_set_error(VD_ERR_ARG, "record: rename to %s failed", dst.c_str());
        ++n;
    }
    if (records_written) *records_written = n;
    return VD_OK;
}
