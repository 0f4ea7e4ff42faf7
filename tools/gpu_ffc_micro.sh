O=${O:-gpurun_out/ffcmicro}; mkdir -p $O
timeout -k 10 300 python -u tools/ffc_micro.py --iters 20 > $O/micro.log 2>&1; rc=$?; cat $O/micro.log | grep -v amdgpu.ids; exit $rc
