import sys; sys.path[:0] = ["/root/repo", "/root/repo/tests"]
import _commit
e, _ = _commit.staged_commit(n_files=200_000, n_dirs=1000)
open(sys.argv[1], "w").write(_commit.to_cli_input(e, {}, 10_000))
