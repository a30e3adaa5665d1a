"""CPU oracle for the wire codec — TEST INFRASTRUCTURE ONLY.

Restates the byte encoding that the reference's `Binary` instances produce for
its message vocabulary:

    newtype Ticket = Ticket Int  deriving Generic;  instance Binary Ticket   Common.hs:20-24
    type Command = String; type Proposal = (Ticket, Command)                 Common.hs:26-30
    data ClientRequest = AskForTicket Ticket | Propose Proposal | Execute Ticket
      deriving Generic; instance Binary ClientRequest                       Common.hs:41-47
    data ServerResponse = Round1OK Ticket (Maybe Proposal) | HaveTicket Ticket
      | Round2Success  deriving Generic; instance Binary ServerResponse      Common.hs:49-55

The instances are GHC.Generics defaults of `binary` (pinned by the reference's
resolver lts-12.18, stack.yaml:20: binary-0.8.5.1, not vendored in
/root/reference).  Its published algorithm (Data.Binary.Generic,
Data.Binary.Class):

* a sum type writes a constructor tag first: Word8 when there are <= 255
  constructors, numbered by `putSum`, which halves the constructor list
  recursively (left half first) — for 3 constructors the tags are 0, 1, 2 in
  declaration order;
* fields follow left to right; a single-constructor newtype (Ticket) writes
  just its field;
* Int = Int64 big-endian (8 bytes); (a, b) = a then b;
  Maybe = Word8 0 | Word8 1 then the value;
  String = [Char] = Int length (8 bytes BE) then each Char as UTF-8.

The message payload is what `sendMessages` hands to `send` as `contentOf m`
(Common.hs:36-39); Cloud Haskell's own envelope (sender ProcessId, type
fingerprint, transport framing) is outside this codec.

Parity status: no GHC in this image, so the bytes are pinned by hand-derived
vectors from the rules above (tests/test_wire.py), not by the reference run.
"""
from __future__ import annotations

import struct
from typing import List, Optional, Tuple

REQUEST, RESPONSE = 0, 1
ASK, PROPOSE, EXECUTE = 0, 1, 2          # ClientRequest tags (declaration order)
R1OK, HAVE, R2S = 0, 1, 2                # ServerResponse tags

OK, E_LENGTH, E_TAG, E_STRING, E_RANGE = 0, 1, 2, 3, 4


def command_string(code: int) -> str:
    """Command code (clientId << 24 | t) -> "c<clientId>.<t>" (Client.hs:202-203)."""
    return "c%d.%d" % (code >> 24, code & 0xFFFFFF)


def _int(v: int) -> bytes:               # Binary Int: Int64 big-endian
    return struct.pack(">q", v)


def _string(s: str) -> bytes:            # Binary [Char]: Int length + UTF-8 chars
    return _int(len(s)) + s.encode("utf-8")


def _proposal(t: int, code: int) -> bytes:   # (Ticket, Command)
    return _int(t) + _string(command_string(code))


def encode(msg: Tuple[int, int, int, int], kind: int) -> bytes:
    """msg = (tag, x, y, z) as pxb_msg: requests x = ticket, z = command;
    responses x = ticket, (y, z) = Round1OK's stored proposal (z == 0: Nothing)."""
    tag, x, y, z = msg
    if kind == REQUEST:
        if tag == ASK:
            return bytes([0]) + _int(x)
        if tag == PROPOSE:
            return bytes([1]) + _proposal(x, z)
        if tag == EXECUTE:
            return bytes([2]) + _int(x)
    else:
        if tag == R1OK:
            mp = bytes([0]) if z == 0 else bytes([1]) + _proposal(y, z)
            return bytes([0]) + _int(x) + mp
        if tag == HAVE:
            return bytes([1]) + _int(x)
        if tag == R2S:
            return bytes([2])
    raise ValueError("bad tag %r" % (tag,))


class _Reader:
    def __init__(self, b: bytes):
        self.b, self.i = b, 0

    def take(self, n: int) -> bytes:
        if self.i + n > len(self.b):
            raise _Err(E_LENGTH)
        r = self.b[self.i:self.i + n]
        self.i += n
        return r

    def int32(self) -> int:
        v = struct.unpack(">q", self.take(8))[0]
        if not -(1 << 31) <= v < (1 << 31):
            raise _Err(E_RANGE)
        return v

    def command(self) -> int:
        """A Command the reference can produce: "c" ++ show id ++ "." ++ show t
        (Client.hs:202-203).  Checked left to right: length range, bytes
        present, grammar (digits without leading zeros), then value range."""
        n = struct.unpack(">q", self.take(8))[0]
        if n < 4 or n > 13:               # "c0.0" .. "c255.16777215"
            raise _Err(E_STRING)
        s = self.take(n)
        if s[0] != ord("c"):
            raise _Err(E_STRING)
        i, vals = 1, []
        for stop in (ord("."), None):     # id digits up to '.', t digits to the end
            j = i
            while j < n and ord("0") <= s[j] <= ord("9"):
                j += 1
            if j == i or (j - i > 1 and s[i] == ord("0")):
                raise _Err(E_STRING)
            vals.append(int(s[i:j]))
            if stop is not None:
                if j >= n or s[j] != stop:
                    raise _Err(E_STRING)
                j += 1
            elif j != n:
                raise _Err(E_STRING)
            i = j
        cid, t = vals
        if cid > 255 or t > 0xFFFFFF:
            raise _Err(E_RANGE)
        return (cid << 24) | t


class _Err(Exception):
    def __init__(self, code):
        self.code = code


def decode(b: bytes, kind: int) -> Tuple[int, Tuple[int, int, int, int]]:
    """Inverse of encode for one framed record: (status, (tag, x, y, z))."""
    r = _Reader(b)
    try:
        tag = r.take(1)[0]
        x = y = z = 0
        if kind == REQUEST:
            if tag in (ASK, EXECUTE):
                x = r.int32()
            elif tag == PROPOSE:
                x = r.int32()
                z = r.command()
            else:
                raise _Err(E_TAG)
        else:
            if tag == R1OK:
                x = r.int32()
                m = r.take(1)[0]
                if m == 1:
                    y = r.int32()
                    z = r.command()
                elif m != 0:
                    raise _Err(E_TAG)
            elif tag == HAVE:
                x = r.int32()
            elif tag != R2S:
                raise _Err(E_TAG)
        if r.i != len(b):
            raise _Err(E_LENGTH)
        return OK, (tag, x, y, z)
    except _Err as e:
        return e.code, (0, 0, 0, 0)


def decode_at(buf: bytes, b: int, e: int, kind: int) -> Tuple[int, Tuple[int, int, int, int]]:
    """Record i of a batch: bytes [b, max(b, e)) of the buffer.  A record that
    reaches past the end of the buffer is a length error (the n_bytes bound
    of pxb_wire_decode); the decode itself is `decode`."""
    e = max(b, e)
    if e > len(buf):
        return E_LENGTH, (0, 0, 0, 0)
    return decode(buf[b:e], kind)


def encode_batch(msgs, kind: int) -> Tuple[bytes, List[int]]:
    out, offs = [], [0]
    for m in msgs:
        e = encode(tuple(int(v) for v in m), kind)   # (tag, x, y, z): signed tickets
        out.append(e)
        offs.append(offs[-1] + len(e))
    return b"".join(out), offs
