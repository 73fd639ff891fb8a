!-----------------------------------------------------------------------
! ed_gpu_driver — Fortran host test driver of the drop-in boundary.
!
! Replays the call sequence of ED_DIAG.f90:139-186 (lanc_method="lanczos")
! and ED_GF_NORMAL.f90:180-195 with the H·v bound through the reference's
! procedure-pointer interface (cc_sparse_HxV, ED_VARS_GLOBAL.f90:48-54):
!   build_Hv_sector   -> ed_gpu_build_sector
!   spHtimesV_cc      => gpuMatVec_cc   (host arrays, PCIe staged)
!   sp_lanc_eigh      -> a host plain-Lanczos loop through spHtimesV_cc,
!                        and the device-resident ed_gpu_lanc_eigh
!   sp_lanc_tridiag   -> ed_gpu_lanc_tridiag
!   delete_Hv_sector  -> ed_gpu_delete_sector (also after a direct build)
!
! usage: ed_gpu_driver Norb Nbath nup ndw [stored|direct]
! Bath: the reference's flat initial bath, init_dmft_bath
! (ED_BATH/dmft_aux.f90:103-135), Nspin=1, U=2, xmu=0, hfmode=T.
!-----------------------------------------------------------------------
program ed_gpu_driver
  use iso_c_binding
  use ED_GPU_HXV
  implicit none

  abstract interface
     subroutine cc_sparse_HxV(Nloc,v,Hv)
       integer                    :: Nloc
       complex(8),dimension(Nloc) :: v
       complex(8),dimension(Nloc) :: Hv
     end subroutine cc_sparse_HxV
  end interface
  procedure(cc_sparse_HxV),pointer :: spHtimesV_cc => null()

  type(ed_params_t)        :: p
  integer                  :: Norb, Nbath, nup, ndw, Nspin, i, Nh, nlanc_h
  integer(c_int64_t)       :: dim8
  integer(c_int32_t)       :: flags, nlanc, vecdim, ng, nconv
  character(len=32)        :: arg
  real(8)                  :: Uloc(3), de, hw, e0_host, e0_dev, resid
  real(8), allocatable     :: e(:,:,:), v(:,:,:), alfa(:), beta(:), a_h(:), b_h(:), eval6(:)
  complex(8), allocatable  :: impHloc(:,:,:,:), vect(:), hv(:), vin(:), evec6(:,:)
  logical                  :: direct

  call get_command_argument(1, arg) ; read(arg,*) Norb
  call get_command_argument(2, arg) ; read(arg,*) Nbath
  call get_command_argument(3, arg) ; read(arg,*) nup
  call get_command_argument(4, arg) ; read(arg,*) ndw
  direct = .false.
  if (command_argument_count() >= 5) then
     call get_command_argument(5, arg)
     direct = (trim(arg) == "direct")
  endif
  Nspin = 1
  Uloc  = [2d0, 0d0, 0d0]
  hw    = 2d0

  ! --- flat bath, dmft_aux.f90:103-135 (no noise: ed_bath_noise_thr=0)
  allocate(e(Nspin,Norb,Nbath), v(Nspin,Norb,Nbath), impHloc(Nspin,Nspin,Norb,Norb))
  impHloc = (0d0,0d0)
  e(:,:,1) = -hw ; e(:,:,Nbath) = hw
  Nh = Nbath/2
  if (mod(Nbath,2)==0 .and. Nbath>=4) then
     de = hw/max(Nh-1,1)
     e(:,:,Nh) = -1.d-3 ; e(:,:,Nh+1) = 1.d-3
     do i = 2, Nh-1
        e(:,:,i) = -hw + (i-1)*de ; e(:,:,Nbath-i+1) = hw - (i-1)*de
     enddo
  elseif (mod(Nbath,2)/=0 .and. Nbath>=3) then
     de = hw/Nh
     e(:,:,Nh+1) = 0d0
     do i = 2, Nh
        e(:,:,i) = -hw + (i-1)*de ; e(:,:,Nbath-i+1) = hw - (i-1)*de
     enddo
  endif
  do i = 1, Nbath
     v(:,:,i) = max(0.1d0, 1d0/sqrt(dble(Nbath)))
  enddo

  call ed_gpu_pack_params(p, Norb, Nspin, Nbath, "normal", "normal", .true., &
       Uloc, 0d0, 0d0, 0d0, 0d0, 0d0, impHloc, e, v)
  call ed_gpu_check(ed_gpu_init(p), "ed_gpu_init")

  ! --- build_Hv_sector(isector): bind spHtimesV_cc
  flags = ED_STORED
  if (direct) flags = ED_DIRECT
  call ed_gpu_check(ed_gpu_build_sector(int(nup,c_int32_t), int(ndw,c_int32_t), flags, dim8), &
       "build_Hv_sector")
  call ed_gpu_check(ed_gpu_vecdim(vecdim), "vecDim_Hv_sector")
  spHtimesV_cc => gpuMatVec_cc
  write(*,"(A,I0,A,I0)") "DIM=", dim8, " VECDIM=", vecdim

  ! --- sp_lanc_eigh through the procedure pointer (host recurrence,
  !     .repo/PLAIN_LANCZOS.f90:87-118), lowest Ritz value by bisection
  allocate(vin(vecdim), hv(vecdim), a_h(300), b_h(301))
  do i = 1, vecdim
     vin(i) = dcmplx(sin(dble(i)), cos(3d0*dble(i)))
  enddo
  call host_lanczos(vecdim, vin, 300, a_h, b_h, nlanc_h)
  e0_host = lowest_eig(nlanc_h, a_h, b_h)
  write(*,"(A,F20.12,A,I0)") "E0_HOST=", e0_host, " NLANC_HOST=", nlanc_h

  ! --- device-resident Lanczos (ground state + Ritz vector)
  allocate(vect(vecdim))
  call ed_gpu_check(ed_gpu_lanc_eigh(512_c_int32_t, 1d-12, 10_c_int32_t, e0_dev, vect, nlanc), &
       "sp_lanc_eigh")
  call spHtimesV_cc(vecdim, vect, hv)
  resid = sqrt(sum(abs(hv - e0_dev*vect)**2))
  write(*,"(A,F20.12,A,I0,A,ES10.3)") "E0_DEV=", e0_dev, " NLANC_DEV=", nlanc, " RESID=", resid

  ! --- sp_lanc_tridiag from the ground state (GF-style seed, same sector)
  allocate(alfa(50), beta(50))
  call ed_gpu_check(ed_gpu_lanc_tridiag(vect, 50_c_int32_t, 1d-13, alfa, beta, ng), "sp_lanc_tridiag")
  write(*,"(A,F20.12,A,I0)") "ALFA1=", alfa(1), " NTRI=", ng

  ! --- sp_eigh (ED_DIAG.f90:145-167): Neigen=6, Nblock=23, tol=1e-12 on the device
  allocate(eval6(6), evec6(vecdim, 6))
  call ed_gpu_check(ed_gpu_eigh(6_c_int32_t, 23_c_int32_t, 512_c_int32_t, 1d-12, vin, eval6, evec6, nconv), &
       "sp_eigh")
  call spHtimesV_cc(vecdim, evec6(:,1), hv)
  write(*,"(A,F20.12,A,F20.12,A,I0,A,ES10.3)") "EIG1=", eval6(1), " EIG6=", eval6(6), " NCONV=", nconv, &
       " EIGRES=", sqrt(sum(abs(hv - eval6(1)*evec6(:,1))**2))

  ! --- MpiStatus=T row split (ED_HAMILTONIAN.f90:55-62 + spMatVec_mpi_cc):
  !     emulate P ranks one after the other, each holding its rows and
  !     applying them to the gathered vector; the assembled product must equal
  !     the serial one bit for bit (same per-row element order)
  call gpuMatVec_cc(vecdim, vin, hv)
  call mpi_rows_check(3, hv)
  call mpi_rows_check(int(dim8) + 2, hv)   ! more ranks than rows: empty ranks

  call ed_gpu_check(ed_gpu_delete_sector(), "delete_Hv_sector")
  call ed_gpu_check(ed_gpu_finalize(), "finalize")
  write(*,"(A)") "DRIVER_OK"

contains

  subroutine mpi_rows_check(nproc, hv_serial)
    integer, intent(in) :: nproc
    complex(8), intent(in) :: hv_serial(:)
    integer(c_int64_t) :: r0, nr, d8
    integer :: rank, nzero, vd
    integer(c_int32_t) :: vdim
    complex(8), allocatable :: hloc(:), hall(:)
    allocate(hall(size(hv_serial)))
    hall = (0d0, 0d0)
    nzero = 0
    do rank = 0, nproc-1
       call ed_gpu_check(ed_gpu_mpi_split(dim8, int(rank, c_int32_t), int(nproc, c_int32_t), r0, nr), "mpi_split")
       call ed_gpu_check(ed_gpu_build_sector_rows(int(nup,c_int32_t), int(ndw,c_int32_t), flags_mpi(), r0, nr, d8), &
            "build_Hv_sector(MPI)")
       call ed_gpu_check(ed_gpu_vecdim(vdim), "vecDim_Hv_sector(MPI)")
       vd = int(vdim)
       if (vd /= int(nr)) stop "vecDim mismatch"
       if (vd == 0) nzero = nzero + 1
       allocate(hloc(max(vd,1)))
       ! the Allgatherv result is the whole vector vin
       call ed_gpu_check(ed_gpu_hxv_mpi(vdim, vin, hloc), "spMatVec_mpi_cc")
       if (vd > 0) hall(int(r0)+1:int(r0)+vd) = hloc(1:vd)
       deallocate(hloc)
    enddo
    write(*,"(A,I0,A,I0,A,L1,A,ES10.3)") "MPI_RANKS=", nproc, " EMPTY_RANKS=", nzero, " MPI_EQUAL=", &
         all(hall == hv_serial), " MPI_RELDEV=", maxval(abs(hall - hv_serial)) / maxval(abs(hv_serial))
  end subroutine mpi_rows_check

  integer(c_int32_t) function flags_mpi()
    flags_mpi = ED_STORED
    if (direct) flags_mpi = ED_DIRECT
  end function flags_mpi

  subroutine host_lanczos(n, v0, nmax, a, b, nl)
    integer, intent(in) :: n, nmax
    complex(8), intent(in) :: v0(n)
    real(8), intent(out) :: a(nmax), b(nmax+1)
    integer, intent(out) :: nl
    complex(8), allocatable :: vv(:), vo(:), tmp(:)
    real(8) :: aa, bb
    integer :: it
    allocate(vv(n), vo(n), tmp(n))
    vv = v0 / sqrt(dble(dot_product(v0, v0)))
    vo = (0d0,0d0) ; bb = 0d0 ; b = 0d0 ; nl = 0
    do it = 1, nmax
       call spHtimesV_cc(n, vv, tmp)
       tmp = tmp - bb*vo
       aa  = dble(dot_product(vv, tmp))
       tmp = tmp - aa*vv
       bb  = sqrt(dble(dot_product(tmp, tmp)))
       vo  = vv
       nl = it ; a(it) = aa ; b(it+1) = bb
       if (abs(bb) < 1d-12) exit
       vv  = tmp/bb
    enddo
  end subroutine host_lanczos

  ! lowest eigenvalue of the symmetric tridiagonal (a, b(2:n)) by Sturm bisection
  real(8) function lowest_eig(n, a, b) result(x)
    integer, intent(in) :: n
    real(8), intent(in) :: a(:), b(:)
    real(8) :: lo, hi, mid, q
    integer :: k, it, cnt
    lo = minval(a(1:n)) - 2d0*maxval(abs(b(2:n+1))) - 1d0
    hi = maxval(a(1:n)) + 2d0*maxval(abs(b(2:n+1))) + 1d0
    do it = 1, 200
       mid = 0.5d0*(lo+hi)
       cnt = 0 ; q = a(1) - mid
       if (q < 0d0) cnt = cnt + 1
       do k = 2, n
          if (q == 0d0) q = 1d-300
          q = (a(k) - mid) - b(k)**2/q
          if (q < 0d0) cnt = cnt + 1
       enddo
       if (cnt >= 1) then
          hi = mid
       else
          lo = mid
       endif
    enddo
    x = 0.5d0*(lo+hi)
  end function lowest_eig

end program ed_gpu_driver
