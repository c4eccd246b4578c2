"""plenum_gpu — MI355X batch Ed25519 verification and quorum tally for
Plenum's request-authentication hot path.

Host-side mirror of the reference interfaces on this path (same class names,
arguments, return values and exceptions), each with a batch entry point that
runs on HIP kernels through the C-ABI library libplenum_verify.so:

  nacl_wrappers   VerifyKey / SigningKey / Signer / Verifier (+ verify_batch)
                  stp_core/crypto/nacl_wrappers.py
  verifier        Verifier / DidVerifier (+ verify_batch)       plenum/common/verifier.py
  client_authn    ClientAuthNr / NaclAuthNr / SimpleAuthNr / CoreAuthMixin /
                  CoreAuthNr (+ verify_batch, authenticate_batch)
                  plenum/server/client_authn.py
  req_authenticator  ReqAuthenticator (+ verify_batch)       plenum/server/req_authenticator.py
  quorums, models Quorums / Commits / Prepares (+ tally_batches)
                  plenum/server/quorums.py, plenum/server/models.py
  serialization, base58, exceptions, constants   the data formats either side

device.py holds the device-resident (torch tensor) entry points; _native.py is
the ctypes binding.  Nothing here verifies on the CPU.
"""
__version__ = '0.1.0'
