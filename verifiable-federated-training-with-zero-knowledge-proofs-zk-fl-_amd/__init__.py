"""MI355X-native Groth16/BN254 prover for the ZK-FL circuits (package root).

Layout: ``csrc/`` HIP kernels + C ABI (built into ``libzkfl.so``), ``zkfl/`` the host-side
mirror of the snarkjs surface (circuit builder, witness program, zkey/wtns formats, ctypes
binding), ``node/`` the N-API binding.  The directory name is not a Python identifier: add it
to ``sys.path`` and ``import zkfl``.
"""
