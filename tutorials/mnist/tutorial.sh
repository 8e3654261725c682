#!/bin/bash
# MNIST tutorial (SNN 784-128-64-10 by default): prepare samples, then alternate
# train_nn / run_nn passes and log the accuracy per pass to ./raw.
# Workflow of the reference's tutorials/mnist/tutorial.bash + opt_mnist.bash,
# non-interactive and offline: MNIST IDX files are taken from $MNIST_DIR (default
# ./mnist: train_images train_labels test_images test_labels); without them pmnist
# writes synthetic MNIST-shaped samples (-g NTR NTE).
#
# Environment: NET=SNN|ANN  HIDDEN="128 64"  PASSES=5  NTR/NTE (synthetic sizes)
#              MODE=batched|online  BATCH=1024  EPOCHS=1  TRAIN=BP|BPM  WORK=./mnist_run
#              FLAGS (extra train_nn/run_nn flags, e.g. "-c" for the CPU engine)
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
BIN=${BIN:-$HERE/../../bin}
for t in pmnist train_nn run_nn; do
  [ -x "$BIN/$t" ] || { echo "missing $BIN/$t (run make first)"; exit 1; }
done
NET=${NET:-SNN}; HIDDEN=${HIDDEN:-"128 64"}; PASSES=${PASSES:-5}
NTR=${NTR:-6000}; NTE=${NTE:-1000}; MODE=${MODE:-batched}; BATCH=${BATCH:-1024}
EPOCHS=${EPOCHS:-1}; TRAIN=${TRAIN:-BP}; WORK=${WORK:-./mnist_run}; MNIST_DIR=${MNIST_DIR:-./mnist}
mkdir -p "$WORK"; WORK=$(cd "$WORK" && pwd)
rm -rf "$WORK/samples" "$WORK/tests"; mkdir -p "$WORK/samples" "$WORK/tests"
PM_FLAGS="-n"; [ "$NET" = SNN ] && PM_FLAGS="-n -s"
if [ -f "$MNIST_DIR/train_images" ]; then
  echo "preparing samples from $MNIST_DIR"
  "$BIN/pmnist" $PM_FLAGS -p "$MNIST_DIR" "$WORK/samples" "$WORK/tests"
else
  echo "no MNIST IDX files in $MNIST_DIR: synthetic samples ($NTR train / $NTE test)"
  "$BIN/pmnist" $PM_FLAGS -g "$NTR" "$NTE" "$WORK/samples" "$WORK/tests"
fi
cd "$WORK"
EXTRA=""
[ "$MODE" = batched ] && EXTRA="[mode] batched
[batch] $BATCH
[epochs] $EPOCHS"
cat > mnist.conf <<!
[name] MNIST
[type] $NET
[init] generate
[seed] 10958
[input] 784
[hidden] $HIDDEN
[output] 10
[train] $TRAIN
[sample_dir] ./samples
[test_dir] ./tests
$EXTRA
!
# continuation conf: start from the previous pass's kernel, reshuffle (seed 0 = time)
sed -e 's/^\[init\].*/[init] kernel.opt/' -e 's/^\[seed\].*/[seed] 0/' mnist.conf > cont_mnist.conf
: > raw
for P in $(seq 1 "$PASSES"); do
  CONF=cont_mnist.conf; [ "$P" = 1 ] && CONF=mnist.conf
  "$BIN/train_nn" -v -v $FLAGS "$CONF" > log 2>&1
  "$BIN/run_nn" -v $FLAGS cont_mnist.conf > results 2>&1
  ACC=$(grep ACCURACY results | awk '{split($2, a, "/"); printf "%.1f", 100 * a[1] / a[2]}')
  LOSS=$(grep -o "loss=[0-9.e+-]*" log | tail -1)
  echo "$P $ACC $LOSS" | tee -a raw
done
echo "All DONE! (pass test-accuracy[%] loss in $WORK/raw)"
