export TMPDIR=/tmp; R=$PWD; cd /tmp
for v in new head; do
  if [ $v = head ]; then cp $R/ab/libgfslam_head.so $R/gf_orb_slam_amd/libgfslam.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/kt_$v -o run --output-format csv -- python3 $R/scripts/kernel_times.py 256 5 > $R/gpurun_out/ktrace_$v.log 2>&1 || exit 3
  python3 - $v <<PY
import csv,glob,collections,sys,json
v=sys.argv[1]
f=glob.glob("/tmp/kt_%s/**/*kernel_trace.csv"%v,recursive=True)[0]
acc=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if int(r.get("Grid_Size_Y","1"))<256: continue
    k=r["Kernel_Name"].replace("(anonymous namespace)::","").split("(")[0]
    acc[k+" "+r.get("Grid_Size_X")].append((int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3)
json.dump({k:(len(x),round(sorted(x)[len(x)//2],1)) for k,x in acc.items()},open("$R/gpurun_out/ktrace_%s.json"%v,"w"),indent=0)
PY
done
