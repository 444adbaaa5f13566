R=$GRAFT_REPO_ROOT
for args in "--mode fwd --n 32 --h 112 --w 112 --c1 144 --c2 144 --k 3 --cout 32" \
            "--mode fwd --n 32 --h 56 --w 56 --c1 240 --c2 240 --k 3 --cout 144" \
            "--mode dgrad --n 32 --h 56 --w 56 --c1 240 --c2 240 --k 3 --cout 144"; do
  for t in -1 20; do
    timeout -k 5 60 python3 $R/tools/conv_micro.py $args --math bf16x3 --tile $t --iters 20 2>&1 | grep -v amdgpu || exit 1
  done
done
