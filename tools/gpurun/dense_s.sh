cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0,'.')
import bench, json
ctx = bench.api.Context(0)
print(json.dumps(bench.bench_dense_s(ctx, n_pt=int(sys.argv[1]) if len(sys.argv) > 1 else 100000)))
ctx.close()
" "$@" 2>&1 | grep -v amdgpu.ids
