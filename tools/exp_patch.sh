R=$GRAFT_REPO_ROOT
for args in "--mode fwd --n 32 --h 224 --w 224 --c1 32 --c2 0 --k 3 --cout 32" \
            "--mode dgrad --n 32 --h 112 --w 112 --c1 144 --c2 144 --k 3 --cout 32" \
            "--mode dgrad --n 32 --h 224 --w 224 --c1 32 --c2 0 --k 3 --cout 32"; do
  for t in 0 2 9 10 20 21 22; do
    timeout -k 5 60 python3 $R/tools/conv_micro.py $args --math bf16x3 --tile $t --iters 20 2>&1 | grep -v amdgpu || exit 1
  done
done
