"""CPU: the product's data-transfer wire codec (libhdfs3_amd/csrc/client/wire.cpp) against
google.protobuf over the reference's own schema.

tests/golden/proto_vectors.json holds messages that google.protobuf encoded, each built the way
the reference builds it (DataTransferProtocolSender.cpp:42-150, PacketHeader.cpp:38-45) or as the
datanode's replies are defined (datatransfer.proto:143-227); tests/golden/make_proto_golden.py made
them from /root/reference/src/proto/*.proto. For every vector:
  * the product's encoder, given the values, writes exactly Google's bytes (and the Send() framing:
    BE16 version 28, the op byte, a varint32 length);
  * the product's decoder reads Google's bytes back to the same values, also with fields it does
    not use and fields unknown to the schema inserted at every nesting level, and large varints;
  * where the decoder enforces required fields, Google's partial serialization without one of them
    is rejected.
The codec is compiled here (g++, host code) with a flat C harness (tests/native/wire_pb_harness.cpp).
tests/dtp.py, the repo's own independent codec, is checked against the same vectors."""
import ctypes
import json
import os
import shutil
import subprocess
import sys

import pytest

from util import REPO

GOLDEN = os.path.join(REPO, "tests", "golden", "proto_vectors.json")
HARNESS = os.path.join(REPO, "tests", "native", "wire_pb_harness.cpp")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    so = tmp_path_factory.mktemp("wirepb") / "libwirepb.so"
    subprocess.run(["g++", "-std=c++17", "-O1", "-shared", "-fPIC", "-I", os.path.join(REPO, "libhdfs3_amd", "csrc"),
                    HARNESS, os.path.join(REPO, "libhdfs3_amd", "csrc", "client", "wire.cpp"), "-o", str(so)],
                   check=True)
    lib = ctypes.CDLL(str(so))
    lib.wh_encode.restype = ctypes.c_long
    lib.wh_encode.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_long]
    lib.wh_decode.restype = ctypes.c_long
    lib.wh_decode.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_long, ctypes.c_char_p, ctypes.c_long]
    return lib


def vectors():
    with open(GOLDEN) as fh:
        return json.load(fh)["vectors"]


def record_text(rec):
    lines = []
    for k, v in rec.items():
        for x in (v if isinstance(v, list) else [v]):
            lines.append(f"{k}={x}")
    return ("\n".join(lines) + "\n").encode()


def parse_record(text):
    out = {}
    for line in text.decode().splitlines():
        k, v = line.split("=", 1)
        val = v if v.startswith("h:") else int(v)
        if k == "status" and k in out:
            out[k] = (out[k] if isinstance(out[k], list) else [out[k]]) + [val]
        else:
            out[k] = val
    return out


def encode(lib, msg, rec):
    buf = ctypes.create_string_buffer(1 << 16)
    n = lib.wh_encode(msg.encode(), record_text(rec), buf, len(buf))
    assert n >= 0, (msg, n)
    return buf.raw[:n]


def decode(lib, msg, data):
    buf = ctypes.create_string_buffer(1 << 16)
    n = lib.wh_decode(msg.encode(), data, len(data), buf, len(buf))
    return None if n == -1 else parse_record(buf.raw[:n])


def canonical(msg, rec):
    """the record the decoder returns for these values (defaults the decoder reports explicitly)"""
    out = dict(rec)
    if msg == "pipeline_ack":
        st = out.get("status", [])
        if len(st) == 1:
            out["status"] = st[0]
        elif not st:
            out.pop("status", None)
    return out


def by_kind():
    kinds = {}
    for v in vectors():
        kinds.setdefault(v["msg"], []).append(v)
    return kinds


KINDS = ["read_block", "block_checksum", "write_block", "packet_header", "block_op_response", "pipeline_ack",
         "client_read_status"]


def test_vectors_cover_every_message():
    kinds = by_kind()
    assert sorted(kinds) == sorted(KINDS)
    assert all(len(kinds[k]) >= 10 for k in KINDS)


@pytest.mark.parametrize("kind", KINDS)
def test_encoder_writes_googles_bytes(harness, kind):
    """wire.cpp's encoders against google.protobuf's serialization of the same values: identical
    bytes (proto2 canonical form, field-number order), and the op framing of Send()."""
    n = 0
    for v in by_kind()[kind]:
        if v.get("decode_only"):
            continue
        got = encode(harness, kind, v["record"])
        want = bytes.fromhex(v.get("frame", v["proto"]))
        assert got == want, (kind, v["record"], got.hex(), want.hex())
        n += 1
    assert n > 0


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("form", ["proto", "unknown"])
def test_decoder_reads_googles_bytes(harness, kind, form):
    """wire.cpp's decoders on google.protobuf's bytes: the same values, with and without fields the
    decoder must skip (schema fields it does not use, fields 1001-1004 of every wire type at every
    nesting level)."""
    for v in by_kind()[kind]:
        data = bytes.fromhex(v[form])
        if kind == "packet_header":  # the decoder takes BE32 packetLen | BE16 protoLen | proto
            frame = bytes.fromhex(v["frame"])
            data = frame[:4] + len(data).to_bytes(2, "big") + data
        got = decode(harness, kind, data)
        assert got is not None, (kind, form, v["record"])
        assert got == canonical(kind, v["record"]), (kind, form)


def test_decoders_reject_missing_required_fields(harness):
    n = 0
    for v in vectors():
        for m in v.get("missing", []):
            assert decode(harness, v["msg"], bytes.fromhex(m)) is None, (v["msg"], m)
            n += 1
    assert n >= 300


def test_packet_header_is_25_proto_bytes_in_31(harness):
    """PacketHeader.cpp:38-45 (CalcPkgHeaderSize): all four fields fixed-width, so every header the
    client writes is 25 proto bytes behind the 6-byte length prefix."""
    for v in by_kind()["packet_header"]:
        if not v.get("decode_only"):
            assert len(bytes.fromhex(v["proto"])) == 25 and len(bytes.fromhex(v["frame"])) == 31


def test_independent_codec_agrees_with_google():
    """tests/dtp.py (the repo's own minimal codec, used by the CPU-side datanode fakes and the
    writer model) builds the same packet headers and READ_BLOCK requests as google.protobuf."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import dtp

    for v in by_kind()["packet_header"]:
        if v.get("decode_only"):
            continue
        r = v["record"]
        assert dtp.packet_header(r["packet_len"], r["offset"], r["seqno"], bool(r["last"]), r["data_len"]) == \
            bytes.fromhex(v["frame"])
    for v in by_kind()["block_op_response"]:
        proto = bytes.fromhex(v["proto"])
        fields = dtp.parse(proto)
        assert fields[1] == [v["record"]["status"]]


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/proto"), reason="reference schema not present")
def test_vectors_regenerate_from_the_reference_schema():
    """Provenance: the committed vectors are exactly what the generator makes from the reference's
    .proto files with google.protobuf (run only where /root/reference exists)."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "tests", "golden", "make_proto_golden.py"), "--check"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
