"""CPU restatement of backuwup's on-disk formats: packfiles and index files.

TEST INFRASTRUCTURE ONLY -- imported by tests/ and bench.py's checks, never by the product
package.  Pure Python over small inputs; the AES-256-GCM / HKDF it needs come from the C oracle
(oracle.py: seal_blob / open_blob, pinned by FIPS-197, the GCM vectors and RFC 5869).

What is restated, with the reference lines it follows:
  - bincode 1.3 `options().with_varint_encoding()` (pack.rs:215, blob_index.rs:193,205): u64
    lengths/ints as varints (< 251 one byte; 251 + u16 LE; 252 + u32 LE; 253 + u64 LE), enum
    tags as varint u32, u8 arrays as raw bytes; deserialization rejects trailing bytes.
  - PackfileHeaderBlob { hash, kind, compression, length, offset } (filesystem/mod.rs:36-43),
    BlobKind / CompressionKind tag order (mod.rs:13-25).
  - Manager::write_packfiles grouping (pack.rs:115-198): queue order; each blob adds
    sealed_len + BLOB_NONCE_SIZE to the blob section; the packfile closes once the section
    reaches PACKFILE_TARGET_SIZE (3 MiB) or PACKFILE_MAX_BLOBS (100 000) blobs (pack.rs:147).
  - Manager::serialize_packfile (pack.rs:200-227): u64 LE header length || AES-GCM(header,
    key = derive_backup_key(b"header"), nonce = packfile id) || (nonce || sealed blob)*.
  - Manager::get_blob (unpack.rs:22-78): the reader, for round trips.
  - BlobIndex::flush / load / counter_to_nonce (blob_index.rs:167-240): index file =
    AES-GCM(bincode varint Vec<(BlobHash, PackfileId)>, key = derive_backup_key(b"index"),
    nonce = u32 LE file number || 0^8).
  - zstd "store" frames: what zstd level 3 emits for incompressible input with the reference's
    settings (pack.rs:58-64: no magic, no checksum, no content size): frame header descriptor
    0x00, window descriptor (wlog - 10) << 3 with wlog = clamp(ceil(log2(len)), 10, 21), then
    raw blocks of <= 128 KiB (3-byte headers, last-block bit).  Pinned against the system
    libzstd by tests/test_pack.py.
"""
import struct

from oracle import oracle

PACKFILE_TARGET_SIZE = 3 * 1024 * 1024   # packfile/mod.rs:25
PACKFILE_MAX_SIZE = 16 * 1024 * 1024     # packfile/mod.rs:27
PACKFILE_MAX_BLOBS = 100_000             # packfile/mod.rs:29
BLOB_NONCE_SIZE = 12                     # shared/src/types.rs
MAX_FILE_ENTRIES = 50_000                # blob_index.rs:16
BLOB_MAX_UNCOMPRESSED_SIZE = 3 * 1024 * 1024  # defaults.rs
KIND_FILE_CHUNK, KIND_TREE = 0, 1
COMPRESSION_NONE, COMPRESSION_ZSTD = 0, 1
ZSTD_BLOCK = 128 * 1024


class FormatError(ValueError):
    """bincode::Error (PackfileError::SerializationError)."""


class CryptoError(ValueError):
    """aes_gcm::Error (PackfileError::CryptoError)."""


# ------------------------------------------------------------------ bincode varint
def varint(v):
    if v < 251:
        return bytes([v])
    if v < 1 << 16:
        return b"\xfb" + struct.pack("<H", v)
    if v < 1 << 32:
        return b"\xfc" + struct.pack("<I", v)
    return b"\xfd" + struct.pack("<Q", v)


def read_varint(buf, pos):
    if pos >= len(buf):
        raise FormatError("unexpected end")
    t = buf[pos]
    if t < 251:
        return t, pos + 1
    size = {251: 2, 252: 4, 253: 8}.get(t)
    if size is None:
        raise FormatError("invalid varint tag %d" % t)
    if pos + 1 + size > len(buf):
        raise FormatError("unexpected end")
    return int.from_bytes(buf[pos + 1:pos + 1 + size], "little"), pos + 1 + size


def header_entry(h, kind, compression, length, offset):
    """bincode varint of one PackfileHeaderBlob (field order of filesystem/mod.rs:36-43)."""
    return bytes(h) + varint(kind) + varint(compression) + varint(length) + varint(offset)


def serialize_header(entries):
    return varint(len(entries)) + b"".join(header_entry(*e) for e in entries)


def deserialize_header(buf):
    n, pos = read_varint(buf, 0)
    out = []
    for _ in range(n):
        if pos + 32 > len(buf):
            raise FormatError("unexpected end")
        h = bytes(buf[pos:pos + 32])
        kind, pos = read_varint(buf, pos + 32)
        comp, pos = read_varint(buf, pos)
        if kind > 1 or comp > 1:
            raise FormatError("invalid enum tag")
        length, pos = read_varint(buf, pos)
        offset, pos = read_varint(buf, pos)
        out.append((h, kind, comp, length, offset))
    if pos != len(buf):
        raise FormatError("trailing bytes")
    return out


# ------------------------------------------------------------------ zstd store frames
def zstd_store_wlog(n):
    wlog = max(1, (n - 1).bit_length()) if n > 1 else 0
    return min(21, max(10, wlog))


def zstd_store(data):
    """Magicless zstd frame of raw blocks (FHD 0x00, window descriptor, blocks of <= 128 KiB)."""
    data = bytes(data)
    out = [bytes([0, (zstd_store_wlog(len(data)) - 10) << 3])]
    nb = max(1, -(-len(data) // ZSTD_BLOCK))
    for k in range(nb):
        blk = data[k * ZSTD_BLOCK:(k + 1) * ZSTD_BLOCK]
        hdr = (len(blk) << 3) | (1 if k == nb - 1 else 0)  # block type 0 = Raw_Block
        out.append(hdr.to_bytes(3, "little") + blk)
    return b"".join(out)


def zstd_store_size(n):
    return 2 + 3 * max(1, -(-n // ZSTD_BLOCK)) + n


# ------------------------------------------------------------------ packfiles
def plan_packfiles(sealed_lens):
    """write_packfiles' grouping (pack.rs:123-148) over the queue of unique blobs: returns
    [(first, count)] per packfile."""
    groups, i, n = [], 0, len(sealed_lens)
    while i < n:
        first, written, count = i, 0, 0
        while i < n:
            written += sealed_lens[i] + BLOB_NONCE_SIZE
            count += 1
            i += 1
            if written >= PACKFILE_TARGET_SIZE or count >= PACKFILE_MAX_BLOBS:
                break
        groups.append((first, count))
    return groups


def session_packfiles(blobs, seeded=()):
    """The reference's write cadence for one packer session, restated literally: blobs =
    [(hash, sealed_len)] in add order (canonical order), seeded = hashes of prior backups.
      add_blob (pack.rs:31-55): a hash already in the index (seeded or written to a packfile) is
        dropped; otherwise it joins the pending queue -- even when an equal blob is still pending;
      trigger_write_if_desired (pack.rs:92-113): rescans the queue for blobs not in the index and
        writes once their sealed bytes reach PACKFILE_TARGET_SIZE or their count PACKFILE_MAX_BLOBS;
      write_packfiles (pack.rs:116-162): drains the whole queue into packfiles, skipping blobs
        that became duplicates, closing each at the target size or blob count (so the last one of
        a drain is a remainder), adding every written blob to the index (blob_index.rs:102-114);
      flush (pack.rs:82-90): one final write_packfiles.
    Returns the packfiles as lists of queue hashes in write order."""
    from collections import deque
    index, pending, out = set(bytes(h) for h in seeded), deque(), []

    def write_packfiles():
        while pending:
            pf, written = [], 0
            while pending:
                h, n = pending.popleft()
                if h in index:
                    continue
                pf.append(h)
                written += n + BLOB_NONCE_SIZE
                index.add(h)
                if written >= PACKFILE_TARGET_SIZE or len(pf) >= PACKFILE_MAX_BLOBS:
                    break
            if pf:
                out.append(pf)

    size = cnt = 0  # the trigger's rescan, kept as a running sum (the index only grows in a drain)
    for h, n in blobs:
        h = bytes(h)
        if h in index:
            continue
        pending.append((h, int(n)))
        size, cnt = size + int(n), cnt + 1
        if len(pending) <= 4096:  # the literal rescan of pack.rs:100-105 where it is affordable
            assert size == sum(b[1] for b in pending if b[0] not in index)
            assert cnt == sum(1 for b in pending if b[0] not in index)
        if size >= PACKFILE_TARGET_SIZE or cnt >= PACKFILE_MAX_BLOBS:
            write_packfiles()
            size = cnt = 0
    write_packfiles()
    return out


def seal_blob_payload(prk, h, nonce, payload):
    """compress_encrypt_blob's encryption (pack.rs:70-80) of an already compressed payload."""
    return oracle.seal_blob(prk, bytes(h), bytes(nonce), bytes(payload))


def serialize_packfile(prk, packfile_id, blobs):
    """blobs: [(hash, kind, nonce, sealed)] -> the packfile bytes (pack.rs:141-146, 200-227)."""
    entries, data, written = [], [], 0
    for h, kind, nonce, sealed in blobs:
        entries.append((h, kind, COMPRESSION_ZSTD, len(sealed), written))
        written += len(sealed) + BLOB_NONCE_SIZE
        data.append(bytes(nonce) + bytes(sealed))
    header = oracle.seal_blob(prk, b"header", bytes(packfile_id), serialize_header(entries))
    buf = struct.pack("<Q", len(header)) + header + b"".join(data)
    if len(buf) > PACKFILE_MAX_SIZE:
        raise AssertionError("bug: violated packfile size limit")
    return buf


def write_packfiles(prk, blobs, packfile_ids):
    """The queue of unique blobs [(hash, kind, nonce, sealed)] -> [(packfile_id, bytes)]."""
    groups = plan_packfiles([len(b[3]) for b in blobs])
    return [(bytes(packfile_ids[g]), serialize_packfile(prk, packfile_ids[g], blobs[f:f + c]))
            for g, (f, c) in enumerate(groups)]


def get_blob(prk, packfile_id, packfile, blob_hash):
    """Manager::get_blob (unpack.rs:22-78) without the decompression: returns (kind, payload)
    of the blob, or raises FormatError/CryptoError where the reference returns an error."""
    if len(packfile) > PACKFILE_MAX_SIZE:
        raise FormatError("PackfileTooLarge")
    hl = struct.unpack_from("<Q", packfile, 0)[0]
    if hl > len(packfile) or hl == 0:
        raise FormatError("InvalidHeaderSize")
    pt = oracle.open_blob(prk, b"header", bytes(packfile_id), bytes(packfile[8:8 + hl]))
    if pt is None:
        raise CryptoError("header")
    base = 8 + hl
    for h, kind, comp, length, offset in deserialize_header(pt):
        if h == bytes(blob_hash):
            at = base + offset
            nonce, sealed = packfile[at:at + 12], packfile[at + 12:at + 12 + length]
            payload = oracle.open_blob(prk, h, bytes(nonce), bytes(sealed))
            if payload is None:
                raise CryptoError("blob")
            return kind, payload
    raise FormatError("IndexHeaderMismatch")


# ------------------------------------------------------------------ index files
def counter_to_nonce(file_num):
    """blob_index.rs:234-240"""
    return struct.pack("<I", file_num) + bytes(8)


def index_plaintext(entries):
    return varint(len(entries)) + b"".join(bytes(h) + bytes(p) for h, p in entries)


def index_file(prk, file_num, entries):
    """BlobIndex::flush (blob_index.rs:202-226): the encrypted file for one items_buf."""
    return oracle.seal_blob(prk, b"index", counter_to_nonce(file_num), index_plaintext(entries))


def parse_index_plaintext(pt):
    n, pos = read_varint(pt, 0)
    if pos + 44 * n > len(pt):
        raise FormatError("unexpected end")
    if pos + 44 * n != len(pt):
        raise FormatError("trailing bytes")
    return [(bytes(pt[pos + 44 * i:pos + 44 * i + 32]), bytes(pt[pos + 44 * i + 32:pos + 44 * i + 44]))
            for i in range(n)]


def load_index(prk, files):
    """BlobIndex::load (blob_index.rs:167-200): files = [(file_num, bytes)] -> items sorted by hash."""
    items = []
    for num, buf in files:
        pt = oracle.open_blob(prk, b"index", counter_to_nonce(num), bytes(buf))
        if pt is None:
            raise CryptoError("index %d" % num)
        items.extend(parse_index_plaintext(pt))
    items.sort(key=lambda e: e[0])
    return items


def push_and_flush(prk, last_file_num, entries):
    """BlobIndex::push (flush at MAX_FILE_ENTRIES, blob_index.rs:151-164) for every entry, then
    the unconditional final flush of Manager::flush (pack.rs:84-90): [(file_num, bytes)]."""
    files, buf, num = [], [], last_file_num
    for e in entries:
        buf.append(e)
        if len(buf) >= MAX_FILE_ENTRIES:
            num += 1
            files.append((num, index_file(prk, num, buf)))
            buf = []
    num += 1
    files.append((num, index_file(prk, num, buf)))
    return files
