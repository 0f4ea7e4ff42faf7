O=gpurun_out/${OUT:-s52}; mkdir -p $O
timeout -k 10 200 python -u tools/restore_micro.py --h 720 --w 1280 > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
timeout -k 10 200 python -u tools/restore_micro.py --h 1080 --w 1920 >> $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
grep -v amdgpu.ids $O/micro.log
