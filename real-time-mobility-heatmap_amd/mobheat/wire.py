"""MongoDB `update` commands straight from a contiguous buffer of pre-encoded statements (the sink of f2).

The reference writes each micro-batch's tiles and latest positions with ``bulk_write(ops, ordered=False)`` in chunks
of 1000 ``UpdateOne`` (heatmap_stream.py:191-196, :230-235).  pymongo sends such a chunk as ONE OP_MSG: section 0 the
command document ``{update: <coll>, ordered: false, $db: <db>}``, section 1 the document sequence ``updates`` -- the
statements ``{q, u, multi: false, upsert: true}`` back to back (pymongo ``message._op_msg``).  The GPU already wrote
those statements back to back (``hm_encode_tile_updates`` / ``hm_encode_position_updates``), so a chunk's section 1 is
one slice of that buffer: this module frames the slice with a 16-B header, the 4-B flags and the small command
document and hands the three pieces to ``socket.sendmsg`` -- no per-statement Python object on the way.

``WireMongoSink`` speaks the protocol itself on a plain TCP connection (``mongodb://host[:port][/db]`` without
credentials, TLS, replica-set or other options, as the reference's default ``MONGO_URI``); ``stream.MongoSink``
(pymongo) stays the sink for every other URI, and sends the same slices as RawBSONDocuments.
"""
import os
import socket
import struct
from urllib.parse import urlparse

import numpy as np

OP_MSG = 2013
BULK_CHUNK = 1000                        # statements per command (reference :191, :230)
MAX_MESSAGE_BYTES = 48_000_000           # MongoDB maxMessageSizeBytes (the hello reply's default)
MAX_WRITE_BATCH = 100_000                # maxWriteBatchSize


def command_doc(collection, db, ordered=False, write_concern=None):
    """BSON of the OP_MSG section-0 command pymongo sends for a bulk of updates (key order as pymongo's)."""
    import bson
    from bson.son import SON
    cmd = SON([("update", collection), ("ordered", bool(ordered))])
    if write_concern:
        cmd["writeConcern"] = write_concern
    cmd["$db"] = db
    return bson.encode(cmd)


def op_msg_parts(request_id, cmd_bson, statements, identifier=b"updates"):
    """The OP_MSG as buffers: [header + flags + section 0, section-1 header, statements] (statements: a bytes-like
    slice of concatenated BSON documents)."""
    seq_len = 4 + len(identifier) + 1 + len(statements)
    total = 16 + 4 + 1 + len(cmd_bson) + 1 + seq_len
    head = struct.pack("<iiiiI", total, request_id, 0, OP_MSG, 0) + b"\x00" + cmd_bson
    sec1 = b"\x01" + struct.pack("<i", seq_len) + identifier + b"\x00"
    return [head, sec1, statements]


def chunks(offsets, max_bytes, max_count=BULK_CHUNK):
    """[(i, j)] statement ranges: at most max_count statements and max_bytes bytes each (a single statement larger
    than max_bytes gets a range of its own: the server then rejects it, as it would pymongo's)."""
    offs = np.asarray(offsets, dtype=np.int64)
    n = offs.size - 1
    out = []
    i = 0
    while i < n:
        j = min(i + max_count, n)
        lim = int(np.searchsorted(offs, offs[i] + max_bytes, side="right")) - 1
        j = max(min(j, lim), i + 1)
        out.append((i, j))
        i = j
    return out


def plain_uri(uri):
    """(host, port, db) when `uri` needs nothing beyond TCP (no credentials, TLS, replica set or options)."""
    u = urlparse(uri)
    if u.scheme != "mongodb" or "@" in u.netloc or "," in u.netloc or u.query or not u.hostname:
        return None
    return u.hostname, u.port or 27017, (u.path or "/").lstrip("/") or None


class WireError(RuntimeError):
    pass


class WireMongoSink:
    """Per-batch connection (the reference opens and closes a MongoClient per batch, :156, :237)."""

    def __init__(self, host, port, db, timeout=60.0):
        self.db = db
        self.host, self.port = host, port
        self._sock = socket.create_connection((host, port), timeout=timeout)
        self._sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._rid = 1

    def _recv_exact(self, n):
        buf = bytearray(n)
        view = memoryview(buf)
        got = 0
        while got < n:
            k = self._sock.recv_into(view[got:], n - got)
            if k == 0:
                raise WireError("connection closed by the server")
            got += k
        return bytes(buf)

    def _reply(self, request_id):
        import bson
        length, _rid, response_to, opcode = struct.unpack("<iiii", self._recv_exact(16))
        body = self._recv_exact(length - 16)
        if opcode != OP_MSG or response_to != request_id:
            raise WireError(f"unexpected reply (opcode {opcode}, responseTo {response_to})")
        flags = struct.unpack_from("<I", body, 0)[0]
        if body[4] != 0:
            raise WireError("reply without a section-0 body")
        end = len(body) - (4 if flags & 1 else 0)   # checksumPresent
        return bson.decode(body[5:end])

    def send_statements(self, collection, buf, lo, hi, n_statements, write_concern=None):
        """One `update` command of the statements in buf[lo:hi) (n_statements of them); returns the reply."""
        rid = self._rid
        self._rid += 1
        parts = op_msg_parts(rid, command_doc(collection, self.db, False, write_concern), memoryview(buf)[lo:hi])
        total = sum(len(p) for p in parts)
        sent = 0
        while sent < total:   # sendmsg may send part of the message
            k = self._sock.sendmsg(parts)
            sent += k
            while parts and k >= len(parts[0]):
                k -= len(parts[0])
                parts = parts[1:]
            if parts and k:
                parts[0] = memoryview(parts[0])[k:]
        return self._reply(rid)

    def update_statements(self, collection, buf, offsets, landed=None):
        """All statements (buf, offsets[n+1]) in unordered commands of <= BULK_CHUNK statements; write errors raise
        pymongo's BulkWriteError like the reference's bulk_write.  landed(upto): the statements are still landing in
        buf (a streamed encode) -- each command is sent once bytes[:its end] are there."""
        offs = np.asarray(offsets, dtype=np.int64)
        base = int(offs[0]) if offs.size else 0
        for i, j in chunks(offs, MAX_MESSAGE_BYTES - 16 * 1024):
            if landed is not None:
                landed(int(offs[j]))
            res = self.send_statements(collection, buf, int(offs[i]) - base, int(offs[j]) - base, j - i)
            raise_write_errors(res)

    def close(self):
        try:
            self._sock.close()
        except OSError:
            pass


def raise_write_errors(res):
    from pymongo.errors import BulkWriteError, OperationFailure
    if not res.get("ok"):
        raise OperationFailure(res.get("errmsg", "update failed"), res.get("code"), res)
    if res.get("writeErrors") or res.get("writeConcernError"):
        raise BulkWriteError({"writeErrors": list(res.get("writeErrors", [])),
                              "writeConcernErrors": [res["writeConcernError"]] if res.get("writeConcernError") else [],
                              "nInserted": 0, "nUpserted": len(res.get("upserted", [])), "nMatched": res.get("n", 0),
                              "nModified": res.get("nModified", 0), "nRemoved": 0, "upserted": res.get("upserted", [])})


def wire_enabled():
    return os.environ.get("MOBHEAT_MONGO_WIRE", "1") != "0"
