"""The restore / merge checks (core/v_latest/index/restore.rs:231-297 should_restore_partial_node,
:300-405 should_restore_file) batched over the ABI (oxen_amd/restore.py), against a per-file
restatement of those functions over the oracle's XXH3-128."""
import os

import numpy as np
import pytest


def _meta_hash(oracle_lib, data: bytes) -> int:
    """maybe_get_metadata_hash(MetadataText) on the oracle: count_lines with chars -> serde_json -> XXH3."""
    lines = 1 + data.count(b"\n")
    chars = sum(1 for b in data if (b & 0xC0) != 0x80)
    return oracle_lib.xxh3_128_int(('{"text":{"num_lines":%d,"num_chars":%d}}' % (lines, chars)).encode())


def _combined(oracle_lib, content: int, meta) -> int:
    """get_combined_hash (hasher.rs:67-80) on the oracle."""
    if meta is None:
        return content
    return oracle_lib.xxh3_128_int(content.to_bytes(16, "little") + int(meta).to_bytes(16, "little"))


def _reference(oracle_lib, path, target, base, mtime_ok, combined, meta_hash):
    """restore.rs:231-297 / :300-405 for one file, restated."""
    if not os.path.exists(path):
        return True
    size = os.stat(path).st_size
    ref = base if base is not None else target
    if mtime_ok and size == ref.num_bytes:
        return True
    h = oracle_lib.xxh3_128_int(open(path, "rb").read())
    if combined:
        h = _combined(oracle_lib, h, meta_hash)
        want, base_h = target.combined_hash, (base.combined_hash if base is not None else None)
    else:
        want, base_h = target.hash, (base.hash if base is not None else None)
    if base is not None:
        if h == want:
            return True
        return h == base_h
    return h == want


def _case(oracle_lib, tmp_path, combined: bool):
    from oxen_amd import hasher
    from oxen_amd.restore import NodeHashes

    rng = np.random.default_rng(7 if combined else 3)
    texts = [b"line one\nline two\n", "café über\n".encode(), b"", b"x" * 70_000]
    old, new, other = {}, {}, {}
    for i, t in enumerate(texts):
        old[i] = t
        new[i] = t + b"changed\n"
        other[i] = bytes(rng.integers(0, 256, 333, dtype=np.uint8))

    def node(data, text_meta):
        c = oracle_lib.xxh3_128_int(data)
        m = _meta_hash(oracle_lib, data) if text_meta else None
        return NodeHashes(hash=c, num_bytes=len(data), combined_hash=_combined(oracle_lib, c, m))

    paths, targets, bases, mt, meta, metah = [], [], [], [], [], []
    k = 0
    # working content x (target, base) x mtime verdict
    for wi, working in enumerate(["old", "new", "other", "missing"]):
        for has_base in (False, True):
            for mtime_ok in (False, True):
                for ti in range(len(texts)):
                    p = tmp_path / f"w{k}.txt"
                    k += 1
                    if working != "missing":
                        p.write_bytes({"old": old, "new": new, "other": other}[working][ti])
                    text_meta = combined and ti % 2 == 0  # half the files carry MetadataText
                    paths.append(str(p))
                    targets.append(node(new[ti], text_meta))
                    bases.append(node(old[ti], text_meta) if has_base else None)
                    mt.append(mtime_ok)
                    meta.append(hasher.TEXT if text_meta else None)
                    data = p.read_bytes() if p.exists() else b""
                    metah.append(_meta_hash(oracle_lib, data) if text_meta else None)
    want = [_reference(oracle_lib, p, t, b, m, combined, mh) for p, t, b, m, mh in zip(paths, targets, bases, mt, metah)]
    return paths, targets, bases, mt, meta, want


@pytest.mark.gpu
@pytest.mark.parametrize("combined", [False, True], ids=["partial_node", "file_node"])
def test_should_restore_matches_the_reference(cuda, oracle_lib, tmp_path, combined):
    """Every branch: missing working file, mtime + size short cut (taken even when the content differs),
    the target's hash, the base's hash, neither; with and without a base node; combined hashes with
    MetadataText counted on the hashing read."""
    from oxen_amd import restore

    paths, targets, bases, mt, meta, want = _case(oracle_lib, tmp_path, combined)
    got = restore.should_restore(paths, targets, bases, mt, combined=combined, file_metadata=meta if combined else None)
    assert got == want
    assert any(want) and not all(want)


@pytest.mark.gpu
def test_should_restore_errors(cuda, oracle_lib, tmp_path):
    """A working path that exists but cannot be read fails the call with hasher.rs's text (the
    reference's `u128_hash_file_contents(..)?`); a directory is such a path (EISDIR on the read)."""
    from oxen_amd import _capi, restore
    from oxen_amd.restore import NodeHashes

    d = tmp_path / "adir"
    d.mkdir()
    f = tmp_path / "ok.txt"
    f.write_bytes(b"hello")
    n = NodeHashes(hash=1, num_bytes=5, combined_hash=1)
    with pytest.raises(_capi.OxenError, match="Could not read file for hashing"):
        restore.should_restore([str(f), str(d)], [n, n], [None, None], [False, False])
    assert restore.should_restore([str(f)], [n], [None], [True]) == [True]  # short cut: no read
    with pytest.raises(_capi.OxenError, match="lengths differ"):
        restore.should_restore([str(f)], [n, n], [None], [True])


def test_should_restore_short_cuts_need_no_device(tmp_path):
    """Missing working files and the mtime + size short cut decide without reading anything (no GPU
    call is made: this runs on the CPU), and argument lengths are checked first."""
    from oxen_amd import _capi, restore
    from oxen_amd.restore import NodeHashes

    f = tmp_path / "same_size.txt"
    f.write_bytes(b"12345")
    t = NodeHashes(hash=1, num_bytes=5, combined_hash=1)
    b = NodeHashes(hash=2, num_bytes=5, combined_hash=2)
    dangling = tmp_path / "dangling"
    dangling.symlink_to(tmp_path / "nowhere")
    got = restore.should_restore([str(tmp_path / "missing"), str(f), str(f), str(f / "x"), str(dangling)],
                                 [t] * 5, [None, b, None, b, None], [False, True, True, False, False])
    # a stat that fails (ENOTDIR, a dangling symlink: exists() follows links) is Path::exists() == false
    assert got == [True] * 5
    for combined in (False, True):
        assert restore.should_restore([], [], [], [], combined=combined) == []
    with pytest.raises(_capi.OxenError, match="lengths differ"):
        restore.should_restore([str(f)], [t], [None, None], [True])


@pytest.mark.gpu
def test_should_restore_first_failing_file_wins(cuda, tmp_path, monkeypatch):
    """per file the reference runs metadata(..)? then the hash (restore.rs:311, :334), so
    the error raised is the first failing FILE's: a hash failure on file 0 beats a stat failure on
    file 1 (the stat failure is a race after exists(), simulated here), and a stat failure on file 0
    beats file 1's hash failure."""
    import os

    from oxen_amd import _capi, restore
    from oxen_amd.restore import NodeHashes

    d = tmp_path / "adir"
    d.mkdir()  # exists, stats, fails its read (EISDIR)
    f = tmp_path / "racy.txt"
    f.write_bytes(b"hello")
    n = NodeHashes(hash=1, num_bytes=5, combined_hash=1)
    real_stat = os.stat

    def stat(p, *a, **k):
        if str(p) == str(f):
            raise FileNotFoundError(2, "gone")
        return real_stat(p, *a, **k)

    import types

    monkeypatch.setattr(restore, "os", types.SimpleNamespace(path=os.path, stat=stat))
    with pytest.raises(_capi.OxenError, match="Could not read file for hashing"):
        restore.should_restore([str(d), str(f)], [n, n], [None, None], [False, False])
    with pytest.raises(_capi.OxenError, match="Could not get file metadata"):
        restore.should_restore([str(f), str(d)], [n, n], [None, None], [False, False])


# ---------------------------------------------------------------- checkout (branches.rs:653-757)
def _checkout_reference(oracle_lib, path, target, frm, t_ok, f_ok, overwrite):
    """branches.rs:653-757 (the File arm of r_restore_missing_or_modified_files) for one file, restated."""
    from oxen_amd import restore as R

    if not os.path.exists(path):
        if frm is not None:
            if frm.hash == target.hash:
                return R.KEEP_DELETED
            if not overwrite:
                return R.CONFLICT
        return R.RESTORE
    size = os.stat(path).st_size
    if t_ok and size == target.num_bytes:
        return R.SKIP
    if frm is not None and f_ok and size == frm.num_bytes:
        return R.RESTORE
    h = oracle_lib.xxh3_128_int(open(path, "rb").read())
    if h == target.hash:
        return R.SKIP
    if frm is not None and h == frm.hash:
        return R.RESTORE
    return R.RESTORE if overwrite else R.CONFLICT


def _checkout_case(oracle_lib, tmp_path):
    from oxen_amd.restore import NodeHashes

    rng = np.random.default_rng(17)
    contents = [b"alpha\n", b"", b"y" * 70_000, bytes(rng.integers(0, 256, 5000, dtype=np.uint8))]

    def node(data):
        return NodeHashes(hash=oracle_lib.xxh3_128_int(data), num_bytes=len(data))

    paths, targets, froms, t_ok, f_ok = [], [], [], [], []
    k = 0
    for ci, base in enumerate(contents):
        tgt, frm_data, other = base + b"target\n", base + b"from!\n", base + b"other edit\n"
        for working in ("target", "from", "other", "missing", "same"):
            for has_from in (False, True):
                for tm, fm in ((False, False), (True, False), (False, True)):
                    p = tmp_path / f"c{k}.bin"
                    k += 1
                    data = {"target": tgt, "from": frm_data, "other": other, "same": None, "missing": None}[working]
                    if data is not None:
                        p.write_bytes(data)
                    paths.append(str(p))
                    targets.append(node(tgt))
                    # "same": deleted, and the from tree holds the target's content (the deletion is kept)
                    froms.append((node(tgt) if working == "same" else node(frm_data)) if has_from else None)
                    t_ok.append(tm)
                    f_ok.append(fm)
    return paths, targets, froms, t_ok, f_ok


@pytest.mark.gpu
@pytest.mark.parametrize("overwrite", [False, True], ids=["abort", "overwrite"])
def test_classify_checkout_matches_the_reference(cuda, oracle_lib, tmp_path, overwrite):
    """Every branch of checkout's File arm: missing (new in the target, deleted with the from tree's own
    content, deleted after a change), the target's and the from node's mtime + size short cuts (taken
    even when the bytes differ), the hash equal to the target's, to the from node's, or neither -- under
    OnConflict::Abort and ::Overwrite; all hashes of one call in one GPU pass."""
    from oxen_amd import restore

    paths, targets, froms, t_ok, f_ok = _checkout_case(oracle_lib, tmp_path)
    got = restore.classify_checkout(paths, targets, froms, t_ok, f_ok, overwrite=overwrite)
    want = [_checkout_reference(oracle_lib, p, t, f, a, b, overwrite)
            for p, t, f, a, b in zip(paths, targets, froms, t_ok, f_ok)]
    assert got == want
    assert set(want) == ({restore.SKIP, restore.RESTORE, restore.KEEP_DELETED} |
                         (set() if overwrite else {restore.CONFLICT}))


@pytest.mark.gpu
def test_classify_checkout_first_failing_file_wins(cuda, tmp_path):
    """A working path that cannot be read (a directory: EISDIR) fails the call with hasher.rs's text,
    the first failing file in walk order; the short cuts before it read nothing."""
    from oxen_amd import _capi, restore
    from oxen_amd.restore import NodeHashes

    d = tmp_path / "adir"
    d.mkdir()
    f = tmp_path / "f.txt"
    f.write_bytes(b"hello")
    n = NodeHashes(hash=1, num_bytes=5)
    assert restore.classify_checkout([str(f)], [n], [None], [True], [False]) == [restore.SKIP]
    with pytest.raises(_capi.OxenError, match="Could not read file for hashing"):
        restore.classify_checkout([str(f), str(d)], [n, NodeHashes(hash=2, num_bytes=1)], [None, None],
                                  [False, False], [False, False])


def test_classify_checkout_short_cuts_need_no_device(tmp_path):
    """Missing files and the two mtime + size short cuts decide without reading anything (no GPU call:
    this runs on the CPU); argument lengths are checked first."""
    from oxen_amd import _capi, restore
    from oxen_amd.restore import NodeHashes

    f = tmp_path / "five.txt"
    f.write_bytes(b"12345")
    t = NodeHashes(hash=1, num_bytes=5)
    same = NodeHashes(hash=1, num_bytes=9)
    diff = NodeHashes(hash=2, num_bytes=5)
    missing = str(tmp_path / "gone")
    got = restore.classify_checkout([missing, missing, missing, str(f), str(f)], [t] * 5,
                                    [None, same, diff, None, diff], [False, False, False, True, False],
                                    [False, False, False, False, True])
    assert got == [restore.RESTORE, restore.KEEP_DELETED, restore.CONFLICT, restore.SKIP, restore.RESTORE]
    assert restore.classify_checkout([missing], [t], [diff], [False], [False], overwrite=True) == [restore.RESTORE]
    with pytest.raises(_capi.OxenError, match="lengths differ"):
        restore.classify_checkout([missing], [t], [None, None], [False], [False])
