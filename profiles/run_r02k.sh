set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02k
mkdir -p $O
timeout -k 10 300 python $R/bench.py --gpus 2 --ydiv 4 --steps 10 --warmup 2 > $O/bench_n2_rehearsal.json 2> $O/bench_n2_rehearsal.err &&
timeout -k 10 100 python -c "import torch; p=torch.cuda.get_device_properties(0); print({a: str(getattr(p,a,None)) for a in ('uuid','pci_bus_id','pci_domain_id','pci_device_id','name','gcnArchName')})" > $O/props.txt 2>&1
