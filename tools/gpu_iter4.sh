# Full-batch path changes: all GPU tests, then the physics production bench.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/it_pytest.log 2>&1 && \
timeout -k 10 400 python tools/physics_bench.py --steps 10 > gpurun_out/physics.log 2>&1 && \
timeout -k 10 300 python tools/physics_bench.py --steps 10 --dtype bf16 --emulate-ranks 4 > gpurun_out/physics_r4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_phys -o phys --output-format csv -- python tools/physics_bench.py --steps 5 --dtype bf16 > gpurun_out/prof_phys.log 2>&1
echo rc=$?
