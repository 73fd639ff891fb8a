!-----------------------------------------------------------------------
! ED_GPU_HXV — iso_c_binding shim between the reference's Fortran call
! sites and the MI355X library libedgpu.so (include/ed_gpu.h).
!
! The reference binds its H·v through the abstract interface
!     cc_sparse_HxV(Nloc,v,Hv)            ED_VARS_GLOBAL.f90:48-54
! and the procedure pointer spHtimesV_cc  ED_VARS_GLOBAL.f90:105,
! set in build_Hv_sector                  ED_HAMILTONIAN.f90:85-101.
! gpuMatVec_cc below has exactly that interface, so a new branch of
! build_Hv_sector can do   spHtimesV_cc => gpuMatVec_cc   and every
! caller (sp_eigh / sp_lanc_eigh / sp_lanc_tridiag in ED_DIAG.f90 and
! ED_GF_*.f90) stays unchanged.  See INTEGRATION.md.
!-----------------------------------------------------------------------
module ED_GPU_HXV
  use iso_c_binding
#ifdef _MPI
  use mpi
#endif
  implicit none
  private

#ifdef _MPI
  ! communicator of the MPI H·v (the reference's MpiComm, ED_VARS_GLOBAL.f90:228-231):
  ! MPI_UNDEFINED until ed_gpu_set_MpiComm sets it, as the reference's MpiComm
  integer, public :: ed_gpu_comm = MPI_UNDEFINED
  public :: ed_gpu_set_MpiComm, ed_gpu_del_MpiComm
#endif

  integer, parameter, public :: ED_MAX_NORB = 3, ED_MAX_NSPIN = 2, ED_MAX_NBATH = 32
  integer, parameter, public :: ED_STORED = 1, ED_DIRECT = 2, ED_REAL = 4

  ! C struct ed_params (include/ed_gpu.h).  C arrays a[I][J][K][L] appear in
  ! Fortran with reversed dimensions (L,K,J,I).
  type, bind(C), public :: ed_params_t
     integer(c_int32_t) :: norb, nspin, nbath, ed_mode, bath_type, hfmode
     real(c_double)     :: uloc(3), ust, jh, jx, jp, xmu
     real(c_double)     :: imphloc_re(ED_MAX_NORB,ED_MAX_NORB,ED_MAX_NSPIN,ED_MAX_NSPIN)
     real(c_double)     :: imphloc_im(ED_MAX_NORB,ED_MAX_NORB,ED_MAX_NSPIN,ED_MAX_NSPIN)
     real(c_double)     :: bath_e(ED_MAX_NBATH,ED_MAX_NORB,ED_MAX_NSPIN)
     real(c_double)     :: bath_v(ED_MAX_NBATH,ED_MAX_NORB,ED_MAX_NSPIN)
     real(c_double)     :: bath_u(ED_MAX_NBATH,ED_MAX_NORB,ED_MAX_NSPIN)
     real(c_double)     :: bath_d(ED_MAX_NBATH,ED_MAX_NORB,ED_MAX_NSPIN)
     real(c_double)     :: bath_h_re(ED_MAX_NBATH,ED_MAX_NORB,ED_MAX_NORB,ED_MAX_NSPIN,ED_MAX_NSPIN)
     real(c_double)     :: bath_h_im(ED_MAX_NBATH,ED_MAX_NORB,ED_MAX_NORB,ED_MAX_NSPIN,ED_MAX_NSPIN)
     real(c_double)     :: bath_vr_re(ED_MAX_NBATH)
     real(c_double)     :: bath_vr_im(ED_MAX_NBATH)
     integer(c_int32_t) :: jz_basis, pad_
  end type ed_params_t

  interface
     integer(c_int) function ed_gpu_init(p) bind(C, name="ed_gpu_init")
       import :: c_int, ed_params_t
       type(ed_params_t), intent(in) :: p
     end function ed_gpu_init
     integer(c_int) function ed_gpu_set_device(dev) bind(C, name="ed_gpu_set_device")
       import :: c_int, c_int32_t
       integer(c_int32_t), value :: dev
     end function ed_gpu_set_device
     integer(c_int) function ed_gpu_build_sector(q1, q2, flags, dim) bind(C, name="ed_gpu_build_sector")
       import :: c_int, c_int32_t, c_int64_t
       integer(c_int32_t), value :: q1, q2, flags
       integer(c_int64_t), intent(out) :: dim
     end function ed_gpu_build_sector
     integer(c_int) function ed_gpu_vecdim(vecdim) bind(C, name="ed_gpu_vecdim")
       import :: c_int, c_int32_t
       integer(c_int32_t), intent(out) :: vecdim
     end function ed_gpu_vecdim
     ! cc_sparse_HxV: Nloc by reference, complex(8) host arrays
     integer(c_int) function ed_gpu_hxv(nloc, v, hv) bind(C, name="ed_gpu_hxv")
       import :: c_int, c_int32_t, c_double_complex
       integer(c_int32_t), intent(in) :: nloc
       complex(c_double_complex), intent(in) :: v(*)
       complex(c_double_complex), intent(out) :: hv(*)
     end function ed_gpu_hxv
     ! MpiStatus=T: rows [row0, row0+nrows) of the sector on this rank
     integer(c_int) function ed_gpu_build_sector_rows(q1, q2, flags, row0, nrows, dim) &
          bind(C, name="ed_gpu_build_sector_rows")
       import :: c_int, c_int32_t, c_int64_t
       integer(c_int32_t), value :: q1, q2, flags
       integer(c_int64_t), value :: row0, nrows
       integer(c_int64_t), intent(out) :: dim
     end function ed_gpu_build_sector_rows
     integer(c_int) function ed_gpu_mpi_split(dim, rank, size, row0, nrows) bind(C, name="ed_gpu_mpi_split")
       import :: c_int, c_int32_t, c_int64_t
       integer(c_int64_t), value :: dim
       integer(c_int32_t), value :: rank, size
       integer(c_int64_t), intent(out) :: row0, nrows
     end function ed_gpu_mpi_split
     ! spMatVec_mpi_cc after the Allgatherv: vin(dim) -> Hv(nloc)
     integer(c_int) function ed_gpu_hxv_mpi(nloc, vin, hv) bind(C, name="ed_gpu_hxv_mpi")
       import :: c_int, c_int32_t, c_double_complex
       integer(c_int32_t), intent(in) :: nloc
       complex(c_double_complex), intent(in) :: vin(*)
       complex(c_double_complex), intent(out) :: hv(*)
     end function ed_gpu_hxv_mpi
     integer(c_int) function ed_gpu_lanc_eigh(nitermax, threshold, ncheck, egs, vect, nlanc) &
          bind(C, name="ed_gpu_lanc_eigh")
       import :: c_int, c_int32_t, c_double, c_double_complex
       integer(c_int32_t), value :: nitermax, ncheck
       real(c_double), value :: threshold
       real(c_double), intent(out) :: egs
       complex(c_double_complex), intent(out) :: vect(*)
       integer(c_int32_t), intent(out) :: nlanc
     end function ed_gpu_lanc_eigh
     integer(c_int) function ed_gpu_lanc_tridiag(v0, nitermax, threshold, alfa, beta, nlanc) &
          bind(C, name="ed_gpu_lanc_tridiag")
       import :: c_int, c_int32_t, c_double, c_double_complex
       complex(c_double_complex), intent(in) :: v0(*)
       integer(c_int32_t), value :: nitermax
       real(c_double), value :: threshold
       real(c_double), intent(out) :: alfa(*), beta(*)
       integer(c_int32_t), intent(out) :: nlanc
     end function ed_gpu_lanc_tridiag
     ! sp_eigh (ARPACK, ED_DIAG.f90:145-167) on the device
     integer(c_int) function ed_gpu_eigh(neigen, nblock, nitermax, tol, v0, evals, evecs, nconv) &
          bind(C, name="ed_gpu_eigh")
       import :: c_int, c_int32_t, c_double, c_double_complex
       integer(c_int32_t), value :: neigen, nblock, nitermax
       real(c_double), value :: tol
       complex(c_double_complex), intent(in) :: v0(*)
       real(c_double), intent(out) :: evals(*)
       complex(c_double_complex), intent(out) :: evecs(*)
       integer(c_int32_t), intent(out) :: nconv
     end function ed_gpu_eigh
     integer(c_int) function ed_gpu_delete_sector() bind(C, name="ed_gpu_delete_sector")
       import :: c_int
     end function ed_gpu_delete_sector
     integer(c_int) function ed_gpu_finalize() bind(C, name="ed_gpu_finalize")
       import :: c_int
     end function ed_gpu_finalize
     type(c_ptr) function ed_gpu_last_error() bind(C, name="ed_gpu_last_error")
       import :: c_ptr
     end function ed_gpu_last_error
     integer(c_size_t) function c_strlen(s) bind(C, name="strlen")
       import :: c_size_t, c_ptr
       type(c_ptr), value :: s
     end function c_strlen
  end interface

  public :: ed_gpu_init, ed_gpu_set_device, ed_gpu_build_sector, ed_gpu_vecdim, ed_gpu_hxv
  public :: ed_gpu_lanc_eigh, ed_gpu_lanc_tridiag, ed_gpu_eigh, ed_gpu_delete_sector, ed_gpu_finalize
  public :: ed_gpu_build_sector_rows, ed_gpu_mpi_split, ed_gpu_hxv_mpi
  public :: gpuMatVec_cc, gpuMatVec_mpi_cc
  public :: ed_gpu_check
  public :: ed_gpu_pack_params

contains

  !> Same interface as cc_sparse_HxV (ED_VARS_GLOBAL.f90:48-54): Hv = H v.
  subroutine gpuMatVec_cc(Nloc, v, Hv)
    integer                    :: Nloc
    complex(8),dimension(Nloc) :: v
    complex(8),dimension(Nloc) :: Hv
    integer(c_int32_t)         :: n
    n = int(Nloc, c_int32_t)
    call ed_gpu_check(ed_gpu_hxv(n, v, Hv), "gpuMatVec_cc")
  end subroutine gpuMatVec_cc

  !> Same interface and contract as spMatVec_mpi_cc (STORED_HxV.f90:147-197):
  !> v and Hv are this rank's Nloc rows; the whole vector is gathered with
  !> MPI_Allgatherv (counts N/P, the last rank N/P + mod(N,P), as the
  !> reference), then the GPU applies the rank's rows of H.  A serial build
  !> (no -D_MPI) is one rank: the gathered vector is v itself.
  subroutine gpuMatVec_mpi_cc(Nloc, v, Hv)
    integer                    :: Nloc
    complex(8),dimension(Nloc) :: v
    complex(8),dimension(Nloc) :: Hv
    complex(8),allocatable     :: vin(:)
    integer                    :: N
#ifdef _MPI
    integer                    :: i, ierr, nproc
    integer,allocatable        :: counts(:), offset(:)
    ! spMatVec_mpi_cc: stop if the communicator was never set (STORED_HxV.f90:157)
    if (ed_gpu_comm == MPI_UNDEFINED) stop "gpuMatVec_mpi_cc ERROR: MpiComm = MPI_UNDEFINED (call ed_gpu_set_MpiComm)"
    call MPI_Comm_size(ed_gpu_comm, nproc, ierr)
    call MPI_Allreduce(Nloc, N, 1, MPI_INTEGER, MPI_SUM, ed_gpu_comm, ierr)
    allocate(counts(0:nproc-1), offset(0:nproc-1))
    counts = N/nproc
    counts(nproc-1) = N/nproc + mod(N, nproc)
    offset = 0
    do i = 1, nproc-1
       offset(i) = offset(i-1) + counts(i-1)
    enddo
    allocate(vin(N))
    call MPI_Allgatherv(v, Nloc, MPI_DOUBLE_COMPLEX, vin, counts, offset, MPI_DOUBLE_COMPLEX, &
         ed_gpu_comm, ierr)
#else
    N = Nloc
    allocate(vin(N))
    vin = v
#endif
    call ed_gpu_check(ed_gpu_hxv_mpi(int(Nloc, c_int32_t), vin, Hv), "gpuMatVec_mpi_cc")
  end subroutine gpuMatVec_mpi_cc

#ifdef _MPI
  !> ed_set_MpiComm (ED_VARS_GLOBAL.f90:295-308): the communicator of gpuMatVec_mpi_cc.
  subroutine ed_gpu_set_MpiComm(comm)
    integer, intent(in) :: comm
    ed_gpu_comm = comm
  end subroutine ed_gpu_set_MpiComm

  !> ed_del_MpiComm: back to MPI_UNDEFINED.
  subroutine ed_gpu_del_MpiComm()
    ed_gpu_comm = MPI_UNDEFINED
  end subroutine ed_gpu_del_MpiComm
#endif

  !> Reference error convention: stop with a message (e.g. STORED_HxV.f90:50).
  subroutine ed_gpu_check(rc, where)
    integer(c_int), intent(in) :: rc
    character(len=*), intent(in) :: where
    type(c_ptr) :: p
    character(kind=c_char), pointer :: msg(:)
    character(len=:), allocatable :: txt
    integer :: i, n
    if (rc == 0) return
    p = ed_gpu_last_error()
    n = int(c_strlen(p))
    call c_f_pointer(p, msg, [n])
    allocate(character(len=n) :: txt)
    do i = 1, n
       txt(i:i) = msg(i)
    enddo
    write(*,"(A,A,A,I0,A,A)") "ED_GPU ERROR in ", where, " (rc=", rc, "): ", txt
    stop 1
  end subroutine ed_gpu_check

  !> Pack the reference's model state (impHloc, dmft_bath components and the
  !> interaction constants) into the C struct.  Arrays use the reference's
  !> shapes: impHloc(Nspin,Nspin,Norb,Norb); e,v,u,d(Nspin,Norb|1,Nbath).
  subroutine ed_gpu_pack_params(p, Norb, Nspin, Nbath, ed_mode, bath_type, hfmode, &
       Uloc, Ust, Jh, Jx, Jp, xmu, impHloc, e, v, u, d)
    type(ed_params_t), intent(out)   :: p
    integer, intent(in)              :: Norb, Nspin, Nbath
    character(len=*), intent(in)     :: ed_mode, bath_type
    logical, intent(in)              :: hfmode
    real(8), intent(in)              :: Uloc(3), Ust, Jh, Jx, Jp, xmu
    complex(8), intent(in)           :: impHloc(:,:,:,:)
    real(8), intent(in)              :: e(:,:,:), v(:,:,:)
    real(8), intent(in), optional    :: u(:,:,:), d(:,:,:)
    integer :: is, js, io, jo, k
    p%norb = Norb ; p%nspin = Nspin ; p%nbath = Nbath
    select case (trim(ed_mode))
    case ("superc") ; p%ed_mode = 1
    case ("nonsu2") ; p%ed_mode = 2
    case default    ; p%ed_mode = 0
    end select
    select case (trim(bath_type))
    case ("hybrid")  ; p%bath_type = 1
    case ("replica") ; p%bath_type = 2
    case default     ; p%bath_type = 0
    end select
    p%hfmode = merge(1, 0, hfmode)
    p%uloc = Uloc ; p%ust = Ust ; p%jh = Jh ; p%jx = Jx ; p%jp = Jp ; p%xmu = xmu
    p%imphloc_re = 0d0 ; p%imphloc_im = 0d0
    p%bath_e = 0d0 ; p%bath_v = 0d0 ; p%bath_u = 0d0 ; p%bath_d = 0d0
    p%bath_h_re = 0d0 ; p%bath_h_im = 0d0 ; p%bath_vr_re = 0d0 ; p%bath_vr_im = 0d0
    p%jz_basis = 0 ; p%pad_ = 0
    do is = 1, Nspin
       do js = 1, Nspin
          do io = 1, Norb
             do jo = 1, Norb
                p%imphloc_re(jo,io,js,is) = dble(impHloc(is,js,io,jo))
                p%imphloc_im(jo,io,js,is) = aimag(impHloc(is,js,io,jo))
             enddo
          enddo
       enddo
    enddo
    do is = 1, Nspin
       do io = 1, size(e,2)
          do k = 1, Nbath
             p%bath_e(k,io,is) = e(is,io,k)
             if (present(d)) p%bath_d(k,io,is) = d(is,io,k)
          enddo
       enddo
       do io = 1, size(v,2)
          do k = 1, Nbath
             p%bath_v(k,io,is) = v(is,io,k)
             if (present(u)) p%bath_u(k,io,is) = u(is,io,k)
          enddo
       enddo
    enddo
  end subroutine ed_gpu_pack_params

end module ED_GPU_HXV
