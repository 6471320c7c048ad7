set -o pipefail
M=tests/test_gpu_multi.py::test_render_multi_async_frames_are_the_ppm_bodies
S=tests/test_gpu_state.py
v() { local tag=$1; shift; timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/t15_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/t15_$tag.log)"; [ $rc -le 1 ] || exit $rc; }
v a "$M[2-None]" $S::test_graph_replayed_small_frames_match_oracle
v b "$M[2-None]" $S::test_replayed_bvh_frames_match_oracle
v c "$M[1-rccl]" $S::test_graph_replayed_small_frames_match_oracle
v d "$M[1-rccl]" $S::test_replayed_bvh_frames_match_oracle
v e "$M[1-None]" $S::test_replayed_bvh_frames_match_oracle $S::test_graph_replayed_small_frames_match_oracle $S::test_render_async_frames_land_in_registered_buffers
