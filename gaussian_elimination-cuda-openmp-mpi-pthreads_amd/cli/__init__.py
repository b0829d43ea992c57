"""Launcher CLIs of the distributed programs (one rank per GPU, torchrun).

The reference's MPI programs are started as `mpirun -np P ./gauss_*_input`
(OpenMP_and_MPI/README.txt); their equivalents here are

  python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 \\
      -m gelim.cli.dist_gauss [-s N | FILE]
  python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 \\
      -m gelim.cli.dist_matmul N

Single-GPU programs are native executables under bin/ (csrc/tools).
"""
