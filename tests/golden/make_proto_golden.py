#!/usr/bin/env python3
"""Generates tests/golden/proto_vectors.json: data-transfer messages encoded by google.protobuf
(the runtime the reference links, here its Python implementation) over the reference's own schema,
read from /root/reference/src/proto/{Security,hdfs,datatransfer}.proto by tests/protoparse.py.

Every message is built the way the reference's sender builds it (DataTransferProtocolSender.cpp:
42-150: BuildBaseHeader sets the block's four fields and the token's four, BuildNodeInfo the six
DatanodeID fields and the location; PacketHeader.cpp:38-45 sets the four packet fields) or, for
what a datanode sends (BlockOpResponseProto, PipelineAckProto), the way its fields are defined
(datatransfer.proto:152-227). Each vector holds:
  record      the harness record (tests/native/wire_pb_harness.cpp) of the message's values
  proto       google.protobuf's serialization (field-number order, the canonical form)
  frame       ops only: BE16 version 28 | u8 op | varint32 length | proto (the Send() framing,
              DataTransferProtocolSender.cpp:42-57); packet headers: BE32 packetLen | BE16 protoLen | proto
  unknown     the same values with fields the decoder must skip: schema fields the product does
              not read (token values, cachingStrategy, DatanodeInfo counters, shortCircuitAccessVersion,
              ...) and fields unknown to the schema (numbers 1001-1004, every wire type) at every
              nesting level
  missing     (where the decoder enforces required fields) the message with one required field
              left out, serialized partially: the decoder must reject it

    python3 tests/golden/make_proto_golden.py [--reference /root/reference] [--check]

--check regenerates and compares with the committed file instead of writing it (exit 1 on a
difference). Deterministic: a fixed seed."""
import argparse
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from protoparse import load_schema  # noqa: E402

OUT = os.path.join(HERE, "proto_vectors.json")
NS = "Hdfs.Internal."
U64_EDGES = [0, 1, 127, 128, 16383, 16384, 2**31 - 1, 2**31, 2**32 - 1, 2**32, 2**35 + 7, 2**56 - 1,
             2**63 - 1, 2**63, 2**64 - 1]
U32_EDGES = [0, 1, 127, 128, 50010, 2**31 - 1, 2**31, 2**32 - 1]
S64_EDGES = [0, 1, -1, 2, -2, 2**31, -(2**31) - 1, 2**62, -(2**62), 2**63 - 1, -(2**63)]
S32_EDGES = [0, 1, -1, 512, 65536, 2**31 - 1, -(2**31)]


def varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def hexs(b):
    return "h:" + b.hex()


class Gen:
    def __init__(self, ref, seed=0x9B0F):
        paths = {n: os.path.join(ref, "src", "proto", n) for n in ("Security.proto", "hdfs.proto", "datatransfer.proto")}
        self.S = load_schema(paths)
        self.X = load_schema(paths, extra_fields=True)
        self.r = random.Random(seed)

    # ---- values -----------------------------------------------------------------------
    def u64(self):
        return self.r.choice(U64_EDGES) if self.r.random() < 0.5 else self.r.getrandbits(self.r.choice([7, 14, 21, 32, 40, 63, 64]))

    def u32(self):
        return self.r.choice(U32_EDGES) if self.r.random() < 0.5 else self.r.getrandbits(self.r.choice([7, 14, 21, 32]))

    def text(self, lo=0, hi=40):
        n = self.r.randint(lo, hi)
        alphabet = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-_.:/"
        s = "".join(self.r.choice(alphabet) for _ in range(n))
        if n and self.r.random() < 0.2:
            s += "é中"  # multi-byte UTF-8
        if self.r.random() < 0.05:
            s = "x" * 200  # a length that needs two varint bytes
        return s

    def blob(self, lo=0, hi=24):
        return bytes(self.r.getrandbits(8) for _ in range(self.r.randint(lo, hi)))

    # ---- message builders (the reference's sender) ---------------------------------------
    def fill_block(self, eb, v):
        eb.poolId, eb.blockId, eb.generationStamp, eb.numBytes = v["pool"], v["block_id"], v["gs"], v["num_bytes"]

    def fill_token(self, tok, real=False):
        if real:
            tok.identifier, tok.password, tok.kind, tok.service = self.blob(1), self.blob(1), self.text(1), self.text(1)
        else:  # a default Token: four empty strings, still set (BuildBaseHeader)
            tok.identifier, tok.password, tok.kind, tok.service = b"", b"", "", ""

    def block_values(self):
        return {"pool": self.text(0, 48), "block_id": self.u64(), "gs": self.u64(), "num_bytes": self.u64()}

    @staticmethod
    def block_record(v):
        return {"pool": hexs(v["pool"].encode()), "block_id": v["block_id"], "gs": v["gs"], "num_bytes": v["num_bytes"]}

    def add_unknown(self, m):
        """set the four out-of-schema fields of an extended-pool message"""
        m.x_unknown_1001 = self.u64()
        m.x_unknown_1002 = self.blob(0, 9)
        m.x_unknown_1003 = self.r.getrandbits(32)
        m.x_unknown_1004 = self.r.getrandbits(64)

    def read_block(self, S, v, extra=False):
        op = S[NS + "OpReadBlockProto"]()
        op.len, op.offset = v["len"], v["offset"]
        op.header.clientName = v["client"]
        self.fill_block(op.header.baseHeader.block, v["block"])
        self.fill_token(op.header.baseHeader.token, real=extra)
        if not v["send_checksums"]:
            op.sendChecksums = False
        if extra:
            op.cachingStrategy.dropBehind = True
            op.cachingStrategy.readahead = self.u64() >> 1
            for m in (op, op.header, op.header.baseHeader, op.header.baseHeader.block, op.header.baseHeader.token,
                      op.cachingStrategy):
                self.add_unknown(m)
        return op

    def write_block(self, S, v, extra=False):
        op = S[NS + "OpWriteBlockProto"]()
        op.latestGenerationStamp, op.minBytesRcvd, op.maxBytesRcvd = v["latest_gs"], v["min_bytes"], v["max_bytes"]
        op.pipelineSize, op.stage = v["pipeline_size"], v["stage"]
        op.header.clientName = v["client"]
        self.fill_block(op.header.baseHeader.block, v["block"])
        self.fill_token(op.header.baseHeader.token, real=extra)
        op.requestedChecksum.bytesPerChecksum, op.requestedChecksum.type = v["bpc"], v["ck_type"]
        for t in v["targets"]:
            info = op.targets.add()
            info.id.hostName, info.id.infoPort, info.id.ipAddr = t["host"], t["info"], t["ip"]
            info.id.ipcPort, info.id.datanodeUuid, info.id.xferPort = t["ipc"], t["uuid"], t["xfer"]
            info.location = t["location"]
            if extra:
                info.id.infoSecurePort = self.u32()
                info.capacity, info.dfsUsed, info.xceiverCount = self.u64(), self.u64(), self.u32()
                info.adminState = 1
                self.add_unknown(info)
                self.add_unknown(info.id)
        if extra:
            op.source.id.ipAddr, op.source.id.hostName, op.source.id.datanodeUuid = "10.0.0.9", "src", "u"
            op.source.id.xferPort, op.source.id.infoPort, op.source.id.ipcPort = 1, 2, 3
            op.cachingStrategy.readahead = 7
            for m in (op, op.header, op.header.baseHeader, op.header.baseHeader.block, op.requestedChecksum):
                self.add_unknown(m)
        return op

    def block_checksum(self, S, v, extra=False):
        op = S[NS + "OpBlockChecksumProto"]()
        self.fill_block(op.header.block, v)
        self.fill_token(op.header.token, real=extra)
        if extra:
            for m in (op, op.header, op.header.block, op.header.token):
                self.add_unknown(m)
        return op

    def packet_header(self, S, v, extra=False):
        h = S[NS + "PacketHeaderProto"]()
        h.offsetInBlock, h.seqno, h.lastPacketInBlock, h.dataLen = v["offset"], v["seqno"], bool(v["last"]), v["data_len"]
        if v.get("sync"):
            h.syncBlock = True
        if extra:
            self.add_unknown(h)
        return h

    def block_op_response(self, S, v, extra=False):
        m = S[NS + "BlockOpResponseProto"]()
        m.status = v["status"]
        if v.get("first_bad_link"):
            m.firstBadLink = v["first_bad_link"]
        if "cr" in v:
            c = v["cr"]
            m.checksumResponse.bytesPerCrc, m.checksumResponse.crcPerBlock = c["bpc"], c["crc_per_block"]
            m.checksumResponse.md5 = c["md5"]
            if c.get("type") is not None:
                m.checksumResponse.crcType = c["type"]
        if "ci" in v:
            c = v["ci"]
            m.readOpChecksumInfo.checksum.type, m.readOpChecksumInfo.checksum.bytesPerChecksum = c["type"], c["bpc"]
            m.readOpChecksumInfo.chunkOffset = c["chunk_offset"]
        if v.get("message"):
            m.message = v["message"]
        if extra:
            m.shortCircuitAccessVersion = self.u32()
            self.add_unknown(m)
            if "cr" in v:
                self.add_unknown(m.checksumResponse)
            if "ci" in v:
                self.add_unknown(m.readOpChecksumInfo)
                self.add_unknown(m.readOpChecksumInfo.checksum)
        return m

    def pipeline_ack(self, S, v, extra=False):
        m = S[NS + "PipelineAckProto"]()
        m.seqno = v["seqno"]
        m.status.extend(v["status"])
        if v["downstream"]:
            m.downstreamAckTimeNanos = v["downstream"]
        if extra:
            self.add_unknown(m)
        return m

    def client_read_status(self, S, v, extra=False):
        m = S[NS + "ClientReadStatusProto"]()
        m.status = v["status"]
        if extra:
            self.add_unknown(m)
        return m

    # ---- cases ----------------------------------------------------------------------------
    STATUSES = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9]

    def cases(self):
        r = self.r
        out = []

        def vec(kind, v, record, frame_fn=None, missing=None):
            proto = getattr(self, kind)(self.S, v).SerializeToString()
            unknown = getattr(self, kind)(self.X, v, extra=True).SerializeToString()
            # the extended-pool bytes are a valid message of the real schema (its unknown fields kept)
            real = type(getattr(self, kind)(self.S, v))()
            real.ParseFromString(unknown)
            assert real.IsInitialized()
            d = {"msg": kind, "record": record, "proto": proto.hex(), "unknown": unknown.hex()}
            if frame_fn:
                d["frame"] = frame_fn(proto).hex()
            if missing is not None:
                d["missing"] = [m.hex() for m in missing]
            out.append(d)

        def op_frame(op):
            return lambda proto: struct.pack(">hB", 28, op) + varint(len(proto)) + proto

        for i in range(40):
            v = {"block": self.block_values(), "client": self.text(0, 60), "offset": self.u64(), "len": self.u64(),
                 "send_checksums": True if i % 8 else False}
            rec = dict(self.block_record(v["block"]), client=hexs(v["client"].encode()), offset=v["offset"],
                       len=v["len"], send_checksums=int(v["send_checksums"]))
            vec("read_block", v, rec, op_frame(81))
        for i in range(30):
            v = self.block_values()
            m = self.block_checksum(self.S, v)
            m.ClearField("header")
            vec("block_checksum", v, self.block_record(v), op_frame(85), missing=[m.SerializePartialToString()])
        for i in range(40):
            ntg = r.choice([0, 1, 2, 3, 5])
            targets = [{"ip": f"10.{r.randint(0, 255)}.{r.randint(0, 255)}.{r.randint(0, 255)}", "host": self.text(0, 30),
                        "uuid": self.text(0, 36), "xfer": self.u32(), "info": self.u32(), "ipc": self.u32(),
                        "location": r.choice(["", "/default-rack", self.text(0, 20)])} for _ in range(ntg)]
            v = {"block": self.block_values(), "client": self.text(0, 60), "targets": targets,
                 "stage": r.choice([0, 1, 2, 3, 4, 5, 6, 7]), "pipeline_size": ntg if i % 5 else self.u32(),
                 "min_bytes": self.u64(), "max_bytes": self.u64(), "latest_gs": self.u64(),
                 "ck_type": r.choice([0, 1, 2]), "bpc": r.choice([512, 1, 4096, 65536, 2**32 - 1, self.u32()])}
            rec = dict(self.block_record(v["block"]), client=hexs(v["client"].encode()))
            for k, t in enumerate(targets):
                for f in ("ip", "host", "uuid", "location"):
                    rec[f"t{k}.{f}"] = hexs(t[f].encode())
                for f in ("xfer", "info", "ipc"):
                    rec[f"t{k}.{f}"] = t[f]
            rec.update(stage=v["stage"], pipeline_size=v["pipeline_size"], min_bytes=v["min_bytes"],
                       max_bytes=v["max_bytes"], latest_gs=v["latest_gs"], ck_type=v["ck_type"], bpc=v["bpc"])
            missing = []
            for fld in ("header", "stage", "pipelineSize", "minBytesRcvd", "maxBytesRcvd", "latestGenerationStamp",
                        "requestedChecksum"):
                m = self.write_block(self.S, v)
                m.ClearField(fld)
                missing.append(m.SerializePartialToString())
            vec("write_block", v, rec, op_frame(80), missing=missing)
        for i in range(60):
            last = i % 6 == 0
            v = {"offset": r.choice(S64_EDGES) if i % 3 == 0 else r.getrandbits(40), "seqno": r.choice(S64_EDGES),
                 "last": int(last), "data_len": 0 if last else r.choice(S32_EDGES), "sync": 0}
            plen = r.choice([4, 4 + 4 * 128 + 65536, 2**31 - 1, r.randint(4, 2**31 - 1)])
            rec = {"packet_len": plen, "offset": v["offset"], "seqno": v["seqno"], "last": v["last"],
                   "data_len": v["data_len"], "sync": 0}
            miss = []
            for fld in ("offsetInBlock", "seqno", "lastPacketInBlock", "dataLen"):
                m = self.packet_header(self.S, v)
                m.ClearField(fld)
                p = m.SerializePartialToString()
                miss.append((struct.pack(">iH", plen, len(p)) + p))
            vec("packet_header", v, rec, lambda proto, plen=plen: struct.pack(">iH", plen, len(proto)) + proto,
                missing=miss)
        for i in range(8):  # syncBlock set (a datanode may send it): decoded, never encoded by a client
            v = {"offset": r.getrandbits(30), "seqno": i, "last": 0, "data_len": 512 * (i + 1), "sync": 1}
            proto = self.packet_header(self.S, v).SerializeToString()
            out.append({"msg": "packet_header", "decode_only": True, "proto": proto.hex(),
                        "frame": (struct.pack(">iH", 4 + 512 * (i + 1) + 4 * (i + 1), len(proto)) + proto).hex(),
                        "unknown": self.packet_header(self.X, v, extra=True).SerializeToString().hex(),
                        "record": {"packet_len": 4 + 512 * (i + 1) + 4 * (i + 1), "offset": v["offset"],
                                   "seqno": i, "last": 0, "data_len": v["data_len"], "sync": 1}})
        for i in range(50):
            v = {"status": r.choice(self.STATUSES)}
            rec = {"status": v["status"]}
            if i % 3 == 1:
                v["first_bad_link"] = self.text(1, 30)
                rec["first_bad_link"] = hexs(v["first_bad_link"].encode())
            if i % 4 == 2:
                v["cr"] = {"bpc": self.u32(), "crc_per_block": self.u64(), "md5": self.blob(16, 16),
                           "type": r.choice([None, 0, 1, 2])}
                rec.update({"cr.bpc": v["cr"]["bpc"], "cr.crc_per_block": v["cr"]["crc_per_block"],
                            "cr.md5": hexs(v["cr"]["md5"])})
                if v["cr"]["type"] is not None:
                    rec["cr.type"] = v["cr"]["type"]
            if i % 2 == 0:
                v["ci"] = {"type": r.choice([0, 1, 2]), "bpc": r.choice([512, 4096, 1, self.u32()]),
                           "chunk_offset": self.u64()}
                rec.update({"ci.type": v["ci"]["type"], "ci.bpc": v["ci"]["bpc"],
                            "ci.chunk_offset": v["ci"]["chunk_offset"]})
            if i % 5 == 3:
                v["message"] = self.text(1, 80)
                rec["message"] = hexs(v["message"].encode())
            m = self.block_op_response(self.S, v)
            m.ClearField("status")
            vec("block_op_response", v, rec, missing=[m.SerializePartialToString()])
        for i in range(50):
            v = {"seqno": r.choice(S64_EDGES + [-1, -1]), "status": [r.choice(self.STATUSES) for _ in range(r.choice([0, 1, 2, 3, 8]))],
                 "downstream": 0 if i % 3 == 0 else self.u64()}
            rec = {"seqno": v["seqno"], "status": list(v["status"]), "downstream": v["downstream"]}
            m = self.pipeline_ack(self.S, v)
            m.ClearField("seqno")
            vec("pipeline_ack", v, rec, missing=[m.SerializePartialToString()])
        for st in self.STATUSES:
            v = {"status": st}
            vec("client_read_status", v, {"status": st}, missing=[b""])
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    g = Gen(a.reference)
    doc = {"generator": "tests/golden/make_proto_golden.py",
           "schema": "reference src/proto/Security.proto, hdfs.proto, datatransfer.proto via tests/protoparse.py",
           "encoder": "google.protobuf (python), SerializeToString / SerializePartialToString",
           "vectors": g.cases()}
    text = json.dumps(doc, indent=0, sort_keys=True) + "\n"
    if a.check:
        same = open(OUT).read() == text
        print("proto vectors match" if same else "proto vectors DIFFER")
        sys.exit(0 if same else 1)
    with open(OUT, "w") as fh:
        fh.write(text)
    print(f"wrote {len(doc['vectors'])} vectors to {OUT}")


if __name__ == "__main__":
    main()
