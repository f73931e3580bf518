for r in 1 2; do for st in 1 4 10 1000; do
ONC_BENCH_TIMED_STRIDE=$st timeout -k 10 200 python bench.py --no-cpu-baseline --no-pcie --c4-leg off > gpurun_out/ab/stride_$st.log 2>&1 || exit $?
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], round(d['value'],1), round(d['ms_per_step']*1e3,1), round(d['ms_per_step_without_kernel_events']*1e3,1), r['launches_timed'], round(r['avg_launch_us'],1))" gpurun_out/ab/stride_$st.log $st
done; done
