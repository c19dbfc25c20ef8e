"""Open failures and read failures are told apart at the ABI.

The reference returns two different errors from hash_small_file_contents (crates/liboxen/src/util/
hasher.rs:126-146): File::open failing gives
    util::hasher::hash_file_contents Could not open file {path:?} {err:?}
(hash_large_file_contents, :150-154, "Could not open file {path:?} due to {err:?}"), a failed
read_to_end gives "Could not read file for hashing". The engine reports OXH_ERR_OPEN / OXH_ERR_IO per
item with the errno (oxh_hash_files_ex and friends), and the mirrors build those texts from it -- no
after-the-fact exists() guess. The expected io::Error Debug text is spelled out here by hand (Rust's
`Os { code, kind, message }` with std's ErrorKind names), not taken from the code under test.
"""
import errno
import os

import pytest

pytestmark = pytest.mark.gpu

ENOENT_DEBUG = 'Os { code: 2, kind: NotFound, message: "No such file or directory" }'
ELOOP_DEBUG = 'Os { code: 40, kind: FilesystemLoop, message: "Too many levels of symbolic links" }'
ENOTDIR_DEBUG = 'Os { code: 20, kind: NotADirectory, message: "Not a directory" }'


@pytest.fixture
def tree(tmp_path):
    ok = tmp_path / "ok.txt"
    ok.write_bytes(b"hello")
    (tmp_path / "dangling").symlink_to(tmp_path / "nowhere")
    (tmp_path / "loop_a").symlink_to(tmp_path / "loop_b")
    (tmp_path / "loop_b").symlink_to(tmp_path / "loop_a")
    (tmp_path / "adir").mkdir()
    return tmp_path


def test_status_and_errno_per_item(cuda, tree):
    from oxen_amd import _capi, hasher

    paths = [str(tree / n) for n in ["ok.txt", "missing", "dangling", "loop_a", "adir"]]
    paths.append(str(tree / ("x" * 300)))  # a component above NAME_MAX
    paths.append(str(tree / "ok.txt" / "x"))  # a file used as a directory
    d, sizes, st, oserr = hasher.hash_files_with_errors_128bit(paths)
    assert st == [0, _capi.OXH_ERR_OPEN, _capi.OXH_ERR_OPEN, _capi.OXH_ERR_OPEN, _capi.OXH_ERR_IO, _capi.OXH_ERR_OPEN,
                  _capi.OXH_ERR_OPEN]
    assert oserr == [0, errno.ENOENT, errno.ENOENT, errno.ELOOP, errno.EISDIR, errno.ENAMETOOLONG, errno.ENOTDIR]
    assert d[0] == hasher.hash_buffer_128bit(b"hello") and all(x is None for x in d[1:])
    # the same through every file entry point that reports errno
    _, _, st2, oserr2 = hasher.hash_files_with_errors_128bit(paths, [5, 0, 0, 0, 4096, 0, 0])
    assert (st2, oserr2) == (st, oserr)
    ds, _, st3 = hasher.hash_files_128bit(paths)
    assert st3 == st and ds[0] == d[0]


def test_reference_messages(cuda, tree):
    from oxen_amd import _capi, hasher

    missing = str(tree / "missing")
    st = os.stat(tree / "ok.txt")
    with pytest.raises(_capi.OxenError) as e:
        hasher.get_hash_given_metadata(missing, st)
    assert str(e.value) == f'util::hasher::hash_file_contents Could not open file "{missing}" {ENOENT_DEBUG}'
    assert e.value.code == _capi.OXH_ERR_OPEN
    loop = str(tree / "loop_a")
    with pytest.raises(_capi.OxenError) as e:
        hasher.get_hash_given_metadata(loop, st)
    assert str(e.value) == f'util::hasher::hash_file_contents Could not open file "{loop}" {ELOOP_DEBUG}'

    class Big:  # metadata of a file >= 1e9 B: the streamed branch's message (hasher.rs:150-154)
        st_size = 2_000_000_000

    with pytest.raises(_capi.OxenError) as e:
        hasher.get_hash_given_metadata(missing, Big())
    assert str(e.value) == f'Could not open file "{missing}" due to {ENOENT_DEBUG}'
    # a directory opens and fails its read (EISDIR): hasher.rs:135-139
    with pytest.raises(_capi.OxenError) as e:
        hasher.hash_file_contents(str(tree / "adir"))
    assert str(e.value) == "Could not read file for hashing" and e.value.code == _capi.OXH_ERR_IO
    # u128_hash_file_contents stats first (util::fs::metadata(path)?, hasher.rs:105): util/fs.rs:593-601 ->
    # OxenError::file_metadata_error (error.rs:1176-1182)
    with pytest.raises(_capi.OxenError) as e:
        hasher.u128_hash_file_contents(missing)
    assert str(e.value) == f'Could not get file metadata: "{missing}" error {ENOENT_DEBUG}'
    with pytest.raises(_capi.OxenError) as e:
        hasher.hash_file_contents(missing)
    assert str(e.value) == f'Could not get file metadata: "{missing}" error {ENOENT_DEBUG}'
    # ENOTDIR (a file used as a directory): an open failure that root cannot bypass, on the GPU box too
    notdir = str(tree / "ok.txt" / "x")
    with pytest.raises(_capi.OxenError) as e:
        hasher.u128_hash_file_contents(notdir)
    assert str(e.value) == f'Could not get file metadata: "{notdir}" error {ENOTDIR_DEBUG}'
    with pytest.raises(_capi.OxenError) as e:
        hasher.get_hash_given_metadata(notdir, st)
    assert str(e.value) == f'util::hasher::hash_file_contents Could not open file "{notdir}" {ENOTDIR_DEBUG}'
    assert e.value.code == _capi.OXH_ERR_OPEN
    # a name with a single quote, bytes outside UTF-8 and a zero-width space: Path's Debug form
    odd_b = os.fsencode(str(tree)) + b"/it's\xff\xfe" + "\u200b".encode()
    with pytest.raises(_capi.OxenError) as e:
        hasher.get_hash_given_metadata(odd_b, st)
    assert str(e.value) == (f'util::hasher::hash_file_contents Could not open file "{tree}/it\\\'s\\xFF\\xFE\\u{{200b}}" '
                            f"{ENOENT_DEBUG}")
    # a path with a quote and a newline: Rust's Debug escapes them
    odd = tree / 'we"ird\nname'
    with pytest.raises(_capi.OxenError) as e:
        hasher.get_hash_given_metadata(str(odd), st)
    assert str(e.value) == (f'util::hasher::hash_file_contents Could not open file "{tree}/we\\"ird\\nname" '
                            f"{ENOENT_DEBUG}")


def test_replaced_by_a_directory_after_the_walk(cuda, tree):
    """The walk saw a 5-byte file; a directory stands at the path when the engine reads it (oxh_hash_files_meta
    semantics: no fstat, the read itself fails with EISDIR) -> a read failure, not an open failure."""
    from oxen_amd import _capi, hasher

    p = tree / "swapped"
    p.write_bytes(b"12345")
    size = os.stat(p).st_size
    p.unlink()
    p.mkdir()
    d, _, st, oserr = hasher.hash_files_with_errors_128bit([str(p), str(tree / "ok.txt")], [size, 5])
    assert st == [_capi.OXH_ERR_IO, 0] and oserr == [errno.EISDIR, 0]
    # and the modified check returns that read's error (fs.rs:1616-1618)
    errs = []
    modified, status, n_hashed = hasher.files_modified([str(p)], [size], [size], [False], [123], os_errors=errs)
    assert status == [_capi.OXH_ERR_IO] and errs == [errno.EISDIR] and n_hashed == 1


def test_permission_denied(cuda, tree):
    from oxen_amd import _capi, hasher

    if os.geteuid() == 0:
        pytest.skip("root opens any file")
    p = tree / "secret"
    p.write_bytes(b"x")
    p.chmod(0)
    try:
        _, _, st, oserr = hasher.hash_files_with_errors_128bit([str(p)])
        assert st == [_capi.OXH_ERR_OPEN] and oserr == [errno.EACCES]
        with pytest.raises(_capi.OxenError) as e:
            hasher.get_hash_given_metadata(str(p), os.stat(p))
        assert str(e.value).endswith('Os { code: 13, kind: PermissionDenied, message: "Permission denied" }')
    finally:
        p.chmod(0o644)


def test_add_files_ex_reports_errno(cuda, tree, tmp_path_factory):
    import numpy as np

    from oxen_amd import _capi, hasher

    root = tmp_path_factory.mktemp("versions")
    paths = [str(tree / "ok.txt"), str(tree / "missing"), str(tree / "adir")]
    table = hasher._PathTable(paths)
    n = len(paths)
    out = np.zeros((n, 2), dtype=np.uint64)
    sizes = np.zeros(n, dtype=np.uint64)
    status = np.zeros(n, dtype=np.int32)
    stored = np.zeros(n, dtype=np.int32)
    oserr = np.full(n, -1, dtype=np.int32)
    ctx = hasher.default_context()
    _capi.check(_capi.lib().oxh_add_files_ex(ctx.handle, table.arg, n, os.fsencode(str(root)),
                                             out.ctypes.data_as(_capi._u64p), sizes.ctypes.data_as(_capi._u64p),
                                             status.ctypes.data_as(_capi._i32p), stored.ctypes.data_as(_capi._i32p),
                                             oserr.ctypes.data_as(_capi._i32p)), "oxh_add_files_ex")
    assert status.tolist() == [0, _capi.OXH_ERR_OPEN, _capi.OXH_ERR_IO]
    assert oserr.tolist() == [0, errno.ENOENT, errno.EISDIR]
    assert stored.tolist() == [1, 0, 0]
    assert os.path.exists(hasher.version_path(str(root), hasher.hash_buffer_128bit(b"hello")))
